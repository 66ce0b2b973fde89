#!/bin/bash
# Round 6 (h): where C4's universes run against each other (residency of the longest universe: CU / XCD co-runners),
# N = 1 and the 8-way shares, and the L2 hit rate of the universe kernels, longest universe alone vs the full set.
set -u
cd /tmp && export TMPDIR=/tmp && cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out
T=${TAG:-r06h}
timeout -k 10 300 python bench.py --workload c4 --steps 2 --warmup 1 --no-cpu-baseline --no-dropin \
  --deterministic-timing 0 > gpurun_out/${T}_c4.log 2>&1 || exit $?
timeout -k 10 400 python bench.py --workload c4 --steps 2 --warmup 1 --place-world 8 --team-width 1 \
  --no-cpu-baseline --no-dropin --deterministic-timing 0 > gpurun_out/${T}_c4_p8.log 2>&1 || exit $?
for m in longest full; do
  extra=""
  [ $m = longest ] && extra="--longest-only --team-width 1"
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc TCC_HIT_sum TCC_MISS_sum SQ_WAVES -d gpurun_out/${T}_tcc_$m \
    -o run --output-format csv -- python3 bench.py --workload c4 $extra --steps 1 --warmup 0 --no-cpu-baseline \
    --no-dropin --deterministic-timing 0 > gpurun_out/${T}_tcc_$m.log 2>&1 || exit $?
done
python3 - <<'PY' > gpurun_out/${T}_tcc_summary.txt
import csv, glob
from collections import defaultdict
for m in ("longest", "full"):
    per = defaultdict(lambda: defaultdict(float))
    for f in glob.glob("gpurun_out/r06h_tcc_%s/*counter_collection.csv" % m):
        for row in csv.DictReader(open(f)):
            if "k_universes" in row["Kernel_Name"]:
                per[(row["Dispatch_Id"], row["Kernel_Name"][:60])][row["Counter_Name"]] += float(row["Counter_Value"])
    for k, v in sorted(per.items()):
        h, mi = v.get("TCC_HIT_sum", 0), v.get("TCC_MISS_sum", 0)
        print(m, k, dict(v), "hit_rate %.3f" % (h / max(h + mi, 1)))
PY
