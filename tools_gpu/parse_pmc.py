"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/run_counter_collection.csv): mean counter value
per dispatch for each kernel (first 40 chars of the name), plus the kernel-trace mean duration."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
# the library the passes profiled (the product build of this tree): bench.py uses the counted bytes only when
# this digest equals the loaded library's
LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "openke-putranse_amd", "openke",
                   "release", "libputranse_hip.so")


def lib_sha256():
    import hashlib
    return hashlib.sha256(open(LIB, "rb").read()).hexdigest() if os.path.exists(LIB) else None
vals = defaultdict(lambda: defaultdict(list))
durs = defaultdict(list)
for f in sorted(glob.glob(os.path.join(root, "p*", "run_counter_collection.csv"))):
    per = defaultdict(float)
    names = {}
    for row in csv.DictReader(open(f)):
        key = (row.get("Dispatch_Id"), row["Counter_Name"])
        per[key] += float(row["Counter_Value"])
        names[row.get("Dispatch_Id")] = row["Kernel_Name"]
    for (did, cn), v in per.items():
        vals[names[did]][cn].append(v)
for f in sorted(glob.glob(os.path.join(root, "p*", "run_kernel_trace.csv"))):
    for row in csv.DictReader(open(f)):
        durs[row["Kernel_Name"]].append(int(row["End_Timestamp"]) - int(row["Start_Timestamp"]))
out = {}
for k, d in vals.items():
    short = k.split("(")[0][-60:]
    out[short] = {cn: sum(v) / len(v) for cn, v in d.items()}
    if durs.get(k):
        out[short]["mean_ns_profiled"] = sum(durs[k]) / len(durs[k])
print(json.dumps(out, indent=1))
if len(sys.argv) > 2 and sys.argv[2].endswith("_uni.json"):   # universe workloads: per-kernel counters only
    json.dump({"lib_sha256": lib_sha256(), "per_kernel": out,
               "method": "rocprofv3 --pmc passes over bench.py --workload (separate passes, --kernel-trace)"},
              open(sys.argv[2], "w"), indent=1)
    print("wrote", sys.argv[2])
    sys.exit(0)

# HBM traffic of one C2 training step for bench.py's roofline.traffic (MI355X_MICROARCH.md §HBM:
# FETCH_SIZE / WRITE_SIZE are kilobytes; on gfx950 FETCH_SIZE counts half the bytes of wide coalesced
# reads, so it is doubled; WRITE_SIZE is exact for streaming stores and float atomics).
# Per step = mean per dispatch of the step kernel + mean per dispatch of the apply kernel + the sampling
# kernels' total over the steps they sampled (argv[3]; bench.py --steps K --warmup W samples W + 3K steps:
# warmup, graph capture run, timed run, measurement run; the isolation re-timing loops sample nothing).
if len(sys.argv) > 2:
    sampled = float(sys.argv[3]) if len(sys.argv) > 3 else None
    # (per chunk of sampled steps: the samplers and the fused path's chunk loss reduction)
    samplers = ("k_sample_csr", "k_scan_counts", "k_sample_sort", "k_advance", "k_sample_part", "k_loss_calls")
    per_step = ("k_step_csr", "k_step_sampled", "k_step_apply", "k_apply")
    def kb(d):
        return 2.0 * sum(d.get("FETCH_SIZE", [])) + sum(d.get("WRITE_SIZE", []))
    total = 0.0
    steps = 0
    parts = {}
    for k, d in vals.items():
        short = k.split("(")[0][-60:]
        n = len(d.get("FETCH_SIZE", []))
        if any(s in k for s in per_step) and n:
            parts[short] = kb(d) / n * 1024.0
            if "k_step" in k:
                steps = max(steps, n)
        elif any(s in k for s in samplers) and n and sampled:
            parts[short] = kb(d) / sampled * 1024.0
    if parts:
        rec = {"lib_sha256": lib_sha256(), "bytes_per_step": sum(parts.values()), "bytes_per_step_by_kernel": parts,
               "step_dispatches_counted": steps, "sampled_steps": sampled,
               "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over bench.py; "
                         "(2 x FETCH_SIZE + WRITE_SIZE) x 1024 B: mean per dispatch of the step and apply "
                         "kernels + the sampling kernels' total / sampled steps",
               "per_kernel": {k.split("(")[0][-60:]: {cn: sum(v) / len(v) for cn, v in d.items()}
                              for k, d in vals.items() if any(s in k for s in samplers + per_step)}}
        json.dump(rec, open(sys.argv[2], "w"), indent=1)
        print("wrote", sys.argv[2], rec["bytes_per_step"])
