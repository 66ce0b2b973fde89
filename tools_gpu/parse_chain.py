"""Summarise a pmc_chain.sh pass: per dispatch of the universe kernel (the longest universe alone), its instruction
counts per training step. The step count and the universe's (bs, dim, ent) come from the bench line of the same run
(its roofline.longest_universe), so bench.py uses the counts only for that universe on this library build."""
import csv
import glob
import hashlib
import json
import os
import sys
from collections import defaultdict

root, out = sys.argv[1], sys.argv[2]
LIB = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "openke-putranse_amd", "openke",
                   "release", "libputranse_hip.so")
line = [ln for ln in open(os.path.join(root, "p1.log")) if ln.startswith("{")][-1]
rec = json.loads(line)
lu = rec["roofline"]["longest_universe"]
per = defaultdict(lambda: defaultdict(float))
for f in glob.glob(os.path.join(root, "p1", "*counter_collection.csv")):
    for row in csv.DictReader(open(f)):
        if "k_universes" not in row["Kernel_Name"]:
            continue
        per[row["Dispatch_Id"]][row["Counter_Name"]] += float(row["Counter_Value"])
disp = list(per.values())
assert disp, "no universe-kernel dispatch in the counters"
mean = {k: sum(d[k] for d in disp) / len(disp) for k in disp[0]}
steps = float(lu["steps"])
res = {"lib_sha256": hashlib.sha256(open(LIB, "rb").read()).hexdigest(),
       "longest": {"bs": lu["bs"], "dim": lu["dim"], "ent": lu["ent"], "steps": lu["steps"]},
       "dispatches": len(disp), "per_dispatch": mean,
       "valu_per_step": mean["SQ_INSTS_VALU"] / steps, "salu_per_step": mean["SQ_INSTS_SALU"] / steps,
       "lds_per_step": mean["SQ_INSTS_LDS"] / steps,
       "vmem_per_step": (mean["SQ_INSTS_VMEM_RD"] + mean["SQ_INSTS_VMEM_WR"]) / steps,
       "waves": mean.get("SQ_WAVES"),
       "wait_fraction": mean["SQ_WAIT_ANY"] / mean["SQ_WAVE_CYCLES"] if mean.get("SQ_WAVE_CYCLES") else None,
       "method": "rocprofv3 --pmc SQ_INSTS_* over bench.py --longest-only --team-width 1 (one workgroup trains the "
                 "workload's longest universe alone); per step = per dispatch / the universe's steps"}
json.dump(res, open(out, "w"), indent=1)
print(json.dumps(res, indent=1))
