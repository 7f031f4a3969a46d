"""Host checks of the kernels' scalar math (csrc/wave.h), compiled with g++ (no GPU)."""
import os
import re
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
WAVE_H = os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd", "csrc", "wave.h")


@pytest.mark.skipif(shutil.which("g++") is None, reason="g++ not available")
def test_log_core_within_one_ulp(tmp_path):
    """log_fast's core (fdlibm reduction + Lg1..Lg7) against libm: < 1 ulp with the exact 1/(2+f),
    < 1.5 ulp with a reciprocal 2 ulps off (the device's v_rcp_f64 + Newton step is closer)."""
    src = open(WAVE_H).read()
    m = re.search(r"template <class Rcp>\n__host__ __device__ __forceinline__ double log_core.*?\n}\n", src, re.S)
    assert m, "log_core not found in wave.h"
    (tmp_path / "log_core_only.h").write_text(m.group(0))
    exe = tmp_path / "check_log"
    subprocess.run(["g++", "-O2", "-I", str(tmp_path), os.path.join(ROOT, "tests", "native", "check_log.cpp"),
                    "-o", str(exe)], check=True)
    r = subprocess.run([str(exe)], capture_output=True, text=True)
    print(r.stdout)
    assert r.returncode == 0, r.stdout


def _economised(n_taylor, keep, odd):
    """Taylor series of sin (odd) / cos (even) to degree n_taylor, Chebyshev-economised on [-1, 1]
    to degrees < keep, in exact rational arithmetic: monomial coefficients and the dropped bound."""
    from fractions import Fraction as F
    from math import factorial
    T = [[F(1)], [F(0), F(1)]]
    for k in range(2, n_taylor + 1):
        a = [F(0)] + [2 * c for c in T[k - 1]]
        b = T[k - 2] + [F(0)] * (len(a) - len(T[k - 2]))
        T.append([x - y for x, y in zip(a, b)])
    mono = [F(0)] * (n_taylor + 1)
    for k in range(1 if odd else 0, n_taylor + 1, 2):
        mono[k] = F((-1) ** (k // 2), factorial(k))
    cheb, rem = [F(0)] * (n_taylor + 1), mono[:]
    for k in range(n_taylor, -1, -1):
        if rem[k]:
            cheb[k] = rem[k] / T[k][k]
            for i, t in enumerate(T[k]):
                rem[i] -= cheb[k] * t
    out = [F(0)] * keep
    for k in range(keep):
        for i, t in enumerate(T[k]):
            if i < keep:
                out[i] += cheb[k] * t
    dropped = sum(abs(c) for c in cheb[keep:]) + F(1, factorial(n_taylor + 1))
    return out, float(dropped)


def test_sincos_small_coefficients_and_accuracy():
    """sincos_small's polynomials (wave.h) are the degree-23 Taylor series economised to degree 15 / 16:
    the coefficients in wave.h are those, rounded to double; truncation <= 5e-20; fma Horner in double
    (emulated exactly) stays within 1.1 ulp of sin / cos on [-1, 1] (the degree-19 / 20 Taylor
    polynomials reached 0.98 / 1.09 ulp on the same grid)."""
    mpmath = pytest.importorskip("mpmath")
    src = open(WAVE_H).read()
    coef = {}
    for name in ("SIN", "COS"):
        m = re.search(r"#define DART_%s_COEFFS (.*?)\n(?!\s)" % name, src, re.S)
        assert m, name
        coef[name] = [float(t) for t in m.group(1).replace("\\", " ").replace("\n", " ").split(",")]
    ps, bs = _economised(23, 16, True)
    pc, bc = _economised(23, 17, False)
    assert bs < 5e-20 and bc < 5e-21
    assert coef["SIN"] == [float(ps[k]) for k in range(3, 16, 2)]
    assert coef["COS"] == [float(pc[k]) for k in range(2, 17, 2)]
    mpmath.mp.dps = 40
    fma = lambda a, b, c: float(mpmath.mpf(a) * mpmath.mpf(b) + mpmath.mpf(c))
    worst_s = worst_c = 0.0
    for i in range(-500, 501):
        x = i / 500.0
        y = x * x
        p = coef["SIN"][-1]
        for c in reversed(coef["SIN"][:-1]):
            p = fma(p, y, c)
        s = fma(x * y, p, x)
        q = coef["COS"][-1]
        for c in reversed(coef["COS"][:-1]):
            q = fma(q, y, c)
        co = fma(y, q, 1.0)
        ts, tc = mpmath.sin(mpmath.mpf(x)), mpmath.cos(mpmath.mpf(x))
        if ts != 0:
            worst_s = max(worst_s, abs(float((mpmath.mpf(s) - ts) / ts)))
        worst_c = max(worst_c, abs(float((mpmath.mpf(co) - tc) / tc)))
    ulp = 2.220446049250313e-16 / 2
    assert worst_s <= 1.1 * ulp and worst_c <= 1.1 * ulp, (worst_s / ulp, worst_c / ulp)


def test_expm1_econ_coefficients_and_accuracy():
    """exp_econ / tanh_econ's P(r) = (e^r - 1 - r) / r^2 (wave.h, LMPC and RMPC) is the degree-19 Taylor P
    economised on |r| <= 0.3467 (the Cody-Waite range ln2 / 2) to degree 10; with fma Horner in
    double (emulated exactly) exp = 1 + r (1 + r P) and expm1 = r + r^2 P stay within 1 / 1.1 ulp,
    as with the degree-11 Taylor P the kernels used before."""
    mpmath = pytest.importorskip("mpmath")
    from fractions import Fraction as F
    from math import factorial
    src = open(WAVE_H).read()
    m = re.search(r"#define DART_EXPM1_COEFFS (.*?)\n(?!\s)", src, re.S)
    assert m
    coef = [float(t) for t in m.group(1).replace("\\", " ").replace("\n", " ").split(",")]
    a = F(3467, 10000)
    n = 19
    T = [[F(1)], [F(0), F(1)]]
    for k in range(2, n + 1):
        u = [F(0)] + [2 * c for c in T[k - 1]]
        v = T[k - 2] + [F(0)] * (len(u) - len(T[k - 2]))
        T.append([x - y for x, y in zip(u, v)])
    mono = [F(1, factorial(k + 2)) * a ** k for k in range(n + 1)]
    cheb, rem = [F(0)] * (n + 1), mono[:]
    for k in range(n, -1, -1):
        cheb[k] = rem[k] / T[k][k]
        for i, t in enumerate(T[k]):
            rem[i] -= cheb[k] * t
    out = [F(0)] * 11
    for k in range(11):
        for i, t in enumerate(T[k]):
            if i < 11:
                out[i] += cheb[k] * t
    assert coef == [float(out[k] / a ** k) for k in range(11)]
    mpmath.mp.dps = 40
    fma = lambda x, y, z: float(mpmath.mpf(x) * mpmath.mpf(y) + mpmath.mpf(z))
    we = wm = 0.0
    for i in range(-600, 601):
        r = 0.3467 * i / 600
        p = coef[-1]
        for c in reversed(coef[:-1]):
            p = fma(p, r, c)
        e, em = fma(fma(p, r, 1.0), r, 1.0), fma(p * r, r, r)
        te, tm = mpmath.exp(mpmath.mpf(r)), mpmath.expm1(mpmath.mpf(r))
        we = max(we, abs(float((mpmath.mpf(e) - te) / te)))
        if tm != 0:
            wm = max(wm, abs(float((mpmath.mpf(em) - tm) / tm)))
    ulp = 2.220446049250313e-16 / 2
    assert we <= 1.0 * ulp and wm <= 1.1 * ulp, (we / ulp, wm / ulp)
