"""Summarise a tools/profile_round.sh run into profiles/<tag>/ (kernel stats + PMC traffic per kernel).

Usage (here, after the gpurun call merged gpurun_out/prof_<tag>):  python tools/summarize_profile.py r01

traffic = (2 * FETCH_SIZE + WRITE_SIZE) per launch, in bytes (KB counters), following
/opt/skills/guides/MI355X_MICROARCH.md: on gfx950 FETCH_SIZE reports half the bytes of wide reads.
"""
import csv
import glob
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TAG = sys.argv[1] if len(sys.argv) > 1 else "r01"
SRC = os.path.join(ROOT, "gpurun_out", f"prof_{TAG}")
DST = os.path.join(ROOT, "profiles", TAG)
os.makedirs(DST, exist_ok=True)

KERNELS = {"pmpc_ipm_kernel": "PMPC (C2, B=18, N=20)", "rmpc_ipm_kernel": "RMPC (C3, B=18, N=20)",
           "lmpc_ipm_kernel": "LMPC (C5, B=18, N=30)", "arm_qp_kernel": "Arm QP (36 arms per launch, n=7)"}
ALGO_BYTES = {"pmpc_ipm_kernel": 18 * 176, "rmpc_ipm_kernel": 18 * (4 + 2 + 14 + 98 + 7 + 2 + 84 + 10 + 14 + 98 + 4) * 8,
              "lmpc_ipm_kernel": 18 * (8 + 2 + 34 + 8 + 22 + 4) * 8,
              "arm_qp_kernel": 36 * (206 + 262 + 7 + 7 + 1 + 1) * 8}   # snapshot + (shared) params read per wave + outputs


# the headline launch of each kernel (B=18 packed 8 blocks per instance; 36 arms): other dispatches
# of the same kernel in the bench (C4, saturation runs) are left out of the per-launch figures
GRID = {"pmpc_ipm_kernel": 18 * 8 * 64, "rmpc_ipm_kernel": 18 * 8 * 64, "lmpc_ipm_kernel": 18 * 8 * 64,
        "arm_qp_kernel": 36 * 64}
# the template instances the headline launches use: round 5, B <= 32 runs the FUSE instantiations of PMPC and
# LMPC (restoration in the solving wave); RMPC's <false> is followed by its queued <true> (~4 us when empty)
STATS_NAME = {"pmpc_ipm_kernel": "pmpc_ipm_kernel<1, true, false, true, false, false, true>",
              "rmpc_ipm_kernel": "rmpc_ipm_kernel<false>",
              "lmpc_ipm_kernel": "lmpc_ipm_kernel<false, true>"}


def short(name):
    for k in KERNELS:
        if k in name:
            return k
    return None


stats = glob.glob(os.path.join(SRC, "trace", "**", "*kernel_stats.csv"), recursive=True)
if stats:
    shutil.copy(stats[0], os.path.join(DST, "kernel_stats.csv"))
summary = {"note": "FETCH_SIZE / WRITE_SIZE from separate rocprofv3 --pmc passes (tools/profile_round.sh), KB; "
                   "traffic_bytes_per_launch = (2*FETCH + WRITE)*1024 (gfx950 FETCH correction, MI355X_MICROARCH.md); "
                   "VGPR_Count / Accum_VGPR_Count / LDS_Block_Size are copied as the kernel trace reports them (they "
                   "do not follow the compiler's arch-VGPR + AGPR split; DESIGN.md §4 quotes -Rpass-analysis counts)",
           "kernels": {}}
per = defaultdict(lambda: defaultdict(list))
meta = {}
for ctr in ("FETCH_SIZE", "WRITE_SIZE"):
    for f in glob.glob(os.path.join(SRC, ctr.split("_")[0].lower(), "**", "*counter_collection.csv"), recursive=True):
        with open(f) as fh:
            for row in csv.DictReader(fh):
                k = short(row.get("Kernel_Name", ""))
                if k is None or row.get("Counter_Name") != ctr or int(row.get("Grid_Size", 0)) != GRID[k]:
                    continue
                if STATS_NAME.get(k, k) not in row.get("Kernel_Name", "") and k != "pmpc_ipm_kernel":
                    continue
                per[k][ctr].append(float(row["Counter_Value"]))
                meta[k] = {"grid_size": int(row.get("Grid_Size", 0)), "VGPR_Count": int(row.get("VGPR_Count", 0)),
                           "Accum_VGPR_Count": int(row.get("Accum_VGPR_Count", 0) or 0),
                           "SGPR_Count": int(row.get("SGPR_Count", 0)), "LDS_Block_Size": int(row.get("LDS_Block_Size", 0)),
                           "Scratch_Size": int(row.get("Scratch_Size", 0) or 0)}
avg = {}
if stats:
    with open(stats[0]) as fh:
        for row in csv.DictReader(fh):
            k = short(row["Name"])
            if k and STATS_NAME.get(k, k) in row["Name"]:
                avg[k] = {"calls_all_grids": int(row["Calls"]), "average_ns_all_grids": float(row["AverageNs"])}
# the per-launch duration of the headline launches alone (the stats line of a template instance also
# counts other batch sizes that use it, e.g. C4's 1152 instances on the PMPC scan build)
traces = glob.glob(os.path.join(SRC, "trace", "**", "*kernel_trace.csv"), recursive=True)
if traces:
    dur = defaultdict(list)
    with open(traces[0]) as fh:
        for row in csv.DictReader(fh):
            k = short(row["Kernel_Name"])
            if k and STATS_NAME.get(k, k) in row["Kernel_Name"] and int(row["Grid_Size_X"]) == GRID[k]:
                dur[k].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
    for k, v in dur.items():
        avg.setdefault(k, {}).update(calls=len(v), average_ns=sum(v) / len(v))
for k, d in per.items():
    fk = sum(d["FETCH_SIZE"]) / max(1, len(d["FETCH_SIZE"]))
    wk = sum(d["WRITE_SIZE"]) / max(1, len(d["WRITE_SIZE"]))
    summary["kernels"][k] = dict(config=KERNELS[k], FETCH_SIZE_KB_mean=fk, FETCH_SIZE_dispatches=len(d["FETCH_SIZE"]),
                                 WRITE_SIZE_KB_mean=wk, WRITE_SIZE_dispatches=len(d["WRITE_SIZE"]),
                                 traffic_bytes_per_launch=(2 * fk + wk) * 1024,
                                 algorithmic_bytes_per_launch=ALGO_BYTES[k], **meta.get(k, {}), **avg.get(k, {}))
if "pmpc_ipm_kernel" in summary["kernels"]:      # bench.py reads the headline kernel's traffic from here
    summary["traffic_bytes_per_launch"] = summary["kernels"]["pmpc_ipm_kernel"]["traffic_bytes_per_launch"]
with open(os.path.join(DST, "pmc_summary.json"), "w") as fh:
    json.dump(summary, fh, indent=1)
print(json.dumps(summary, indent=1))
