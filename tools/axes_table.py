"""Tabulate tools/bench_axes.py JSON lines: one row per file, ms per axis set.
usage: python tools/axes_table.py FILE..."""
import json
import sys

AXES = ["(0,)", "(1,)", "(2,)", "(0, 1)", "(1, 2)", "(0, 2)"]
print("%-44s" % "file" + "".join("%9s" % a for a in AXES))
for f in sys.argv[1:]:
    line = [x for x in open(f) if x.startswith("{")][-1]
    r = json.loads(line)["results"]
    print("%-44s" % f.split("/")[-1][:44] + "".join("%9s" % (r[a].get("ms", "-") if a in r else "-") for a in AXES))
