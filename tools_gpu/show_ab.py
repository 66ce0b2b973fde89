"""Summarise ab_libs.sh logs: ms per step and the longest universe's phase cycles per build and workload."""
import glob
import json
import re
import sys

tag = sys.argv[1] if len(sys.argv) > 1 else "ab"
rows = {}
for f in sorted(glob.glob("gpurun_out/%s_*_c?_?.log" % tag)):
    m = re.match(r".*/%s_(.+)_(c\d)_(\d)\.log" % re.escape(tag), f)
    lib, wl, rep = m.groups()
    txt = open(f).read()
    ms = None
    for line in txt.splitlines():
        if line.startswith("{"):
            ms = json.loads(line)["ms_per_step"]
    top = re.search(r"universe-prof span ([\d.]+) Mcyc steps (\d+) bs (\d+) D (\d+).*presample (\d+)\s+A (\d+)\s+B (\d+)", txt)
    rows.setdefault((wl, lib), []).append((ms, top.groups() if top else None))
for (wl, lib), v in sorted(rows.items()):
    print(wl, lib.ljust(8), " ".join("%.1f" % x[0] if x[0] else "-" for x in v), "| longest:",
          " ; ".join("%s Mcyc bs %s D %s pre %s A %s B %s" % (t[0], t[2], t[3], t[4], t[5], t[6]) for _, t in v if t))
