"""Summarise a zero-sign profile directory (tools/gpu/r05_zs3.sh output):
per query, the end-to-end median per zero fraction and the pyas kernels'
average durations."""
import csv
import json
import os
import sys

d = sys.argv[1]
names = sorted({f.rsplit("_z", 1)[0] for f in os.listdir(d) if f.endswith(".json") and "_z" in f})
for n in names:
    line = [n]
    for z in ("0", "0.02", "0.5"):
        f = os.path.join(d, f"{n}_z{z}.json")
        if not os.path.exists(f):
            continue
        ms = json.load(open(f))["ms_median"]
        ks = list(csv.DictReader(open(os.path.join(d, f"{n}_z{z}_kernel_stats.csv"))))
        ks = [k for k in ks if "pyas::" in k["Name"]]
        tot = sum(float(k["TotalDurationNs"]) for k in ks) / max(int(k["Calls"]) for k in ks) / 1e3
        top = max(ks, key=lambda k: float(k["TotalDurationNs"]))
        line.append(f"z{z}: {ms:.3f} ms (pyas {tot:.0f} us; top {top['Name'].split('(')[0].replace('void pyas::', '')[:40]} "
                    f"{float(top['AverageNs']) / 1e3:.0f} us)")
    print("\n   ".join(line))
for f in sorted(os.listdir(d)):
    if f.endswith(".json") and "_z" not in f:
        print(f, json.load(open(os.path.join(d, f)))["ms_median"])
