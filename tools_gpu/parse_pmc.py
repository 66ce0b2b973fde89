"""Summarise rocprofv3 --pmc passes (gpurun_out/pmc/p*/run_counter_collection.csv): mean counter value
per dispatch for each kernel (first 40 chars of the name), plus the kernel-trace mean duration."""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

root = sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/pmc"
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

# HBM traffic of one C2 training step for bench.py's roofline.traffic (MI355X_MICROARCH.md §HBM:
# FETCH_SIZE / WRITE_SIZE are kilobytes; on gfx950 FETCH_SIZE counts half the bytes of wide coalesced
# reads, so it is doubled; WRITE_SIZE is exact for streaming stores and float atomics)
if len(sys.argv) > 2:
    step_kernels = ("k_sample_csr", "k_scan_counts", "k_sample_sort", "k_advance", "k_step_csr", "k_step_sampled", "k_apply")
    fetch = write = 0.0
    steps = 0
    for k, d in vals.items():
        if not any(s in k for s in step_kernels):
            continue
        fetch += sum(d.get("FETCH_SIZE", []))
        write += sum(d.get("WRITE_SIZE", []))
        if "k_step_csr" in k or "k_step_sampled" in k:
            steps = max(steps, len(d.get("FETCH_SIZE", [])))
    if steps:
        rec = {"bytes_per_step": (2.0 * fetch + write) * 1024.0 / steps,
               "fetch_kb_per_step_raw": fetch / steps, "write_kb_per_step": write / steps,
               "steps_counted": steps,
               "method": "rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE in separate passes over bench.py; "
                         "(2 x FETCH_SIZE + WRITE_SIZE) x 1024 B summed over k_sample_sort, k_advance, k_sample_csr, k_scan_counts, "
                         "k_step_csr, k_apply_buf dispatches / k_step_csr dispatches",
               "per_kernel": {k.split("(")[0][-60:]: {cn: sum(v) / len(v) for cn, v in d.items()}
                              for k, d in vals.items() if any(s in k for s in step_kernels)}}
        json.dump(rec, open(sys.argv[2], "w"), indent=1)
        print("wrote", sys.argv[2], rec["bytes_per_step"])
