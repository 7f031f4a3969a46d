"""Bit-for-bit comparison of two tools/ab_variant.py dumps: python tools/ab_compare.py a.npz b.npz"""
import sys

import numpy as np

a, b = np.load(sys.argv[1]), np.load(sys.argv[2])
same = {k: bool(np.array_equal(a[k], b[k], equal_nan=True)) for k in ("u0", "st", "it", "f")}
du = float(np.nanmax(np.abs(a["u0"] - b["u0"])))
print("bit-identical" if all(same.values()) else "DIFFERENT", same, f"max|du0| {du:.3e}",
      f"iters equal {np.mean(a['it'] == b['it']) * 100:.3f} %", f"status equal {np.mean(a['st'] == b['st']) * 100:.3f} %")
