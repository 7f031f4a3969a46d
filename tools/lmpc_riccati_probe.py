"""Inputs of C5 stress instance i (tools/lmpc_mismatch.py numbering) for tools/lmpc_riccati_probe.c, then runs it.
Usage: python tools/lmpc_riccati_probe.py <i> [seed0=100000]"""
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "oracle"), os.path.join(ROOT, "dart-dual-arm-non-prehensile-manipulation_amd")]
import oracle_lib  # noqa: E402
from dart_mpc.workload import lmpc_batch  # noqa: E402

i = int(sys.argv[1]); seed0 = int(sys.argv[2]) if len(sys.argv) > 2 else 100000
D = lmpc_batch(1, seed0=seed0 + i // 18)
b = i % 18
x = np.concatenate([D["state"][b], D["u_prev"][b], D["pvec"][b], D["target"][b], oracle_lib.LMPC_PRM_DEFAULT])
path = "/tmp/lmpc_probe_in.bin"
x.astype(np.float64).tofile(path)
exe = "/tmp/lmpc_riccati_probe"
subprocess.run(["gcc", "-O2", "-o", exe, os.path.join(ROOT, "tools", "lmpc_riccati_probe.c"), "-lm", "-lquadmath"], check=True)
subprocess.run([exe, path], check=True)
