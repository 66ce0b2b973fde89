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
