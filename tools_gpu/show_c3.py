"""Print the universe fields of bench lines: s_per_step and the class launches' overlap (measurement tooling)."""
import json
import sys

for f in sys.argv[1:]:
    line = [ln for ln in open(f) if ln.startswith("{")][-1]
    d = json.loads(line)
    u = d.get("pu_c3", d)
    cl = u.get("class_launches") or {}
    print("%-40s lib %s s/step %.2f ms overlap %s span %s launches %s" % (
        f.split("/")[-1], (d.get("roofline", {}).get("lib_sha256") or "")[:8], 1e3 * (u.get("s_per_step") or
        d.get("ms_per_step", 0) / 1e3), round(cl.get("overlap", 0), 2), round(cl.get("span_ms", 0), 2),
        cl.get("launches")))
