"""Print the c3_slab / c3_stride query lines of a bench.py JSON output."""
import json
import sys

for path in sys.argv[1:]:
    b = json.load(open(path))
    print(path, "value", b["value"], "frac", b["roofline"]["frac"])
    for k, v in b.get("extra", {}).items():
        if not k.startswith("c3_"):
            continue
        for q in v.get("queries", []):
            print(f"  {k:9s} {q['index']:18s} {str(q['axis']):6s} {q['method']:5s} {q['ms_per_step']:7.4f} ms "
                  f"frac {q['frac']:.4f}" + (f" touched {q['frac_touched_lines']:.4f}" if 'frac_touched_lines' in q else ""))
