"""Per-launch durations and the idle gaps between consecutive launches of one kernel, from a
rocprofv3 --kernel-trace CSV (tools/trace_gaps.sh).  Usage: python tools/kernel_gaps.py <csv> <substr>"""
import csv
import sys

import numpy as np

rows = [r for r in csv.DictReader(open(sys.argv[1])) if sys.argv[2] in r["Kernel_Name"]]
rows.sort(key=lambda r: int(r["Start_Timestamp"]))
s = np.array([int(r["Start_Timestamp"]) for r in rows], dtype=np.float64)
e = np.array([int(r["End_Timestamp"]) for r in rows], dtype=np.float64)
d = (e - s) / 1e3
gap = (s[1:] - e[:-1]) / 1e3
print(f"{sys.argv[2]}: {len(rows)} launches, duration mean {d.mean():.1f} us (median {np.median(d):.1f}, "
      f"min {d.min():.1f}, max {d.max():.1f}); gap to the previous launch median {np.median(gap):.1f} us, "
      f"mean {gap.mean():.1f} us")
