"""Summarise a PT_KAPPA_LOG (tests/helpers.py assert_step_close records, one per compared table of a teacher-forced
step) into the committed profiles/*_parity_bound_summary.json: per test file the comparisons, largest error,
largest ratio (error over the bound's rounding term), largest allowed bound and exemptions, plus the worst records.

  python tools_gpu/kappa_summary.py LOG.jsonl OUT.json "source text"
"""
import json
import sys


def main():
    log, out, source = sys.argv[1], sys.argv[2], sys.argv[3]
    recs = [json.loads(ln) for ln in open(log) if ln.strip()]
    by = {}
    for r in recs:
        f = r["test"].split("::")[0].split("/")[-1]
        b = by.setdefault(f, {"comparisons": 0, "max_abs_err": 0.0, "max_ratio": -1e9, "max_allowed": 0.0,
                              "tie_rows": 0, "noise": 0, "compared_elements": 0, "ill_conditioned": 0,
                              "max_err_well_conditioned": 0.0})
        b["comparisons"] += 1
        b["max_abs_err"] = max(b["max_abs_err"], r.get("max_err", 0.0))
        b["max_ratio"] = max(b["max_ratio"], r.get("ratio", 0.0))
        b["max_allowed"] = max(b["max_allowed"], r.get("max_allowed", 0.0))
        b["tie_rows"] += r.get("tie_rows", 0)
        b["noise"] += r.get("noise", 0)
        b["compared_elements"] += r.get("compared", 0)
        b["ill_conditioned"] += r.get("ill_conditioned", 0)
        b["max_err_well_conditioned"] = max(b["max_err_well_conditioned"],
                                            r.get("max_err_well_conditioned", r.get("max_err", 0.0)))
    top = sorted(recs, key=lambda r: -r.get("ratio", 0.0))[:12]
    summ = {"source": source, "comparisons": len(recs), "by_file": by,
            "max_ratio": max((r.get("ratio", 0.0) for r in recs), default=0.0),
            "max_abs_err": max((r.get("max_err", 0.0) for r in recs), default=0.0),
            "max_allowed": max((r.get("max_allowed", 0.0) for r in recs), default=0.0),
            "ill_conditioned": sum(r.get("ill_conditioned", 0) for r in recs),
            "max_err_well_conditioned": max((r.get("max_err_well_conditioned", r.get("max_err", 0.0)) for r in recs),
                                            default=0.0),
            "largest_ratios": top}
    json.dump(summ, open(out, "w"), indent=1)
    print(json.dumps({k: summ[k] for k in ("comparisons", "max_ratio", "max_abs_err", "max_allowed", "ill_conditioned",
                                           "max_err_well_conditioned")}))


if __name__ == "__main__":
    main()
