// Host check of log_core (wave.h) against libm: max error in ulps over a log-uniform sample and
// [1e-12, 2), with the exact 1 / (2 + f) and with a reciprocal perturbed by 2 ulps (the device
// uses v_rcp_f64 + one Newton step).  Built and run by tests/test_math.py, which extracts
// log_core from csrc/wave.h into log_core_only.h (the header itself needs hip_runtime.h).
#include <cmath>
#include <cstdio>
#include <random>
#define __host__
#define __device__
#define __forceinline__ inline
using std::fma;
double frcp(double x) { return 1.0 / x; }
#include "log_core_only.h"

struct Exact { double operator()(double f) const { return 1.0 / (2.0 + f); } };
struct Perturbed { double operator()(double f) const { return std::nextafter(std::nextafter(1.0 / (2.0 + f), 1.0), 1.0); } };

template <class R>
double max_ulp(R r) {
    std::mt19937_64 g(1);
    double worst = 0;
    for (int i = 0; i < 4000000; ++i) {
        const double x = (i % 2) ? std::exp(std::uniform_real_distribution<double>(-700, 700)(g))
                                 : std::uniform_real_distribution<double>(1e-12, 2.0)(g);
        int e;
        const double m = std::frexp(x, &e);
        const double v = log_core(m, e, r), ref = std::log(x);
        if (ref == 0) continue;
        const long double d = std::fabs((long double)v - logl((long double)x));
        worst = std::fmax(worst, (double)(d / std::ldexp(1.0L, std::ilogb(ref) - 52)));
    }
    return worst;
}
int main() {
    const double a = max_ulp(Exact()), b = max_ulp(Perturbed());
    std::printf("log_core max error: %.3f ulp (exact reciprocal), %.3f ulp (reciprocal +2 ulp)\n", a, b);
    return (a < 1.0 && b < 1.5) ? 0 : 1;
}
