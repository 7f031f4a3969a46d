"""Summarise a tools/pmc_sq.sh run into profiles/<tag>/sq_summary.json (SQ instruction / cycle counters).

Usage (here, after the gpurun call merged gpurun_out/sq_<tag>):  python tools/summarize_sq.py r01

Means over the headline launches of each kernel (grid filter: B = 18 packed 8 blocks per instance,
36 arms); per-instance figures divide by the working waves (the XCD packing launches 8 blocks per
instance and 7 of them exit at once).  SQ_WAVE_CYCLES and SQ_ACTIVE_INST_VALU count 4-cycle units.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TAG = sys.argv[1] if len(sys.argv) > 1 else "r01"
SRC = os.path.join(ROOT, "gpurun_out", f"sq_{TAG}")
DST = os.path.join(ROOT, "profiles", TAG, "sq_summary.json")

# label: (kernel-name prefix, grid size of the headline launch, working waves per launch)
# (B <= 32 launches run the fused instantiations: <..., FUSE = true>, restoration in the solving wave)
KERNELS = {"PMPC C2": ("void dartmpc::pmpc_ipm_kernel<1, true, false, true, false", 9216, 18),
           "RMPC C3": ("void dartmpc::rmpc_ipm_kernel<false", 9216, 18),
           "LMPC C5": ("void dartmpc::lmpc_ipm_kernel<false", 9216, 18),
           "arm QP": ("void dartmpc::arm_qp_kernel<7>", 2304, 36)}

files = sorted(glob.glob(os.path.join(SRC, "**", "*counter_collection.csv"), recursive=True))
if not files:
    sys.exit(f"no counter_collection.csv under {SRC}")
vals = defaultdict(lambda: defaultdict(dict))     # label -> (pass, dispatch) -> counter -> value
for fi, fn in enumerate(files):        # the SQ pass and the MFMA pass (tools/pmc_sq.sh)
    with open(fn) as fh:
        for row in csv.DictReader(fh):
            for label, (prefix, grid, _) in KERNELS.items():
                if row["Kernel_Name"].startswith(prefix) and int(row["Grid_Size"]) == grid:
                    d = vals[label][(fi, row["Dispatch_Id"])]
                    d[row["Counter_Name"]] = d.get(row["Counter_Name"], 0.0) + float(row["Counter_Value"])

out = {"note": "rocprofv3 --pmc SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_WAIT_INST_ANY "
               "SQ_ACTIVE_INST_VALU SQ_INSTS_SMEM, and a second pass SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_WAVES "
               "SQ_BUSY_CYCLES (tools/pmc_sq.sh, tools/summarize_sq.py), means over the headline "
               "launches; per-instance figures divide by the working waves (18 / 36; the XCD packing launches 8 "
               "blocks per instance, 7 exit at once); SQ_WAVE_CYCLES and SQ_ACTIVE_INST_VALU count 4-cycle units",
       "kernels": {}}
for label, disp in vals.items():
    names = sorted({c for d in disp.values() for c in d})
    # per counter: the mean over the dispatches of the pass that collected it
    mean = {c: (sum(d[c] for d in disp.values() if c in d) / sum(1 for d in disp.values() if c in d)) for c in names}
    w = KERNELS[label][2]
    per = {"valu_insts": mean["SQ_INSTS_VALU"] / w, "salu_insts": mean["SQ_INSTS_SALU"] / w,
           "lds_insts": mean["SQ_INSTS_LDS"] / w, "wave_cycles": 4 * mean["SQ_WAVE_CYCLES"] / w,
           "valu_active_cycles": 4 * mean["SQ_ACTIVE_INST_VALU"] / w}
    per["valu_busy_frac"] = per["valu_active_cycles"] / per["wave_cycles"]
    per["cycles_per_valu_inst"] = per["wave_cycles"] / per["valu_insts"]
    if "SQ_VALU_MFMA_BUSY_CYCLES" in mean:
        # matrix-core busy cycles per working wave and as a fraction of the wave's cycles (0: no MFMA issued)
        per["mfma_busy_cycles"] = mean["SQ_VALU_MFMA_BUSY_CYCLES"] / w
        per["mfma_busy_frac"] = per["mfma_busy_cycles"] / per["wave_cycles"]
    out["kernels"][label] = {"dispatches": len(disp), "counters_mean": mean, "per_instance": per}
with open(DST, "w") as fh:
    json.dump(out, fh, indent=1)
for label, k in out["kernels"].items():
    p = k["per_instance"]
    print(f"{label:8s} valu {p['valu_insts']:9.0f}  cycles {p['wave_cycles']:9.0f}  busy {p['valu_busy_frac']:.2f}  "
          f"cyc/valu {p['cycles_per_valu_inst']:.2f}")
