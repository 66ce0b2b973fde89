"""Print the bench lines of the given logs compactly (value, us/step, per-kernel us)."""
import json
import sys

for f in sys.argv[1:]:
    for line in open(f):
        if line.startswith('{"metric"'):
            d = json.loads(line)
            r = d["roofline"]
            print("%-28s %.3fG  %.2f us/step  frac %.3f  %s" % (f.split("/")[-1], d["value"] / 1e9, d["ms_per_step"] * 1e3,
                  r["frac"], {k: round(v * 1e3, 2) for k, v in r.get("ms_per_kernel", {}).items()}))
        elif "part-prof" in line:
            print("   ", line.strip())
