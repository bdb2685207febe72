"""Print the top pyas kernels of every *_kernel_stats.csv in a directory,
with the end-to-end median of the matching .json when there is one."""
import csv
import glob
import json
import os
import sys

d = sys.argv[1]
for f in sorted(glob.glob(d + "/*_kernel_stats.csv")):
    rows = list(csv.DictReader(open(f)))
    tag = os.path.basename(f).replace("_kernel_stats.csv", "")
    j = f.replace("_kernel_stats.csv", ".json")
    e2e = json.load(open(j)).get("ms_median") if os.path.exists(j) else None
    print(tag, e2e)
    for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:5]:
        if "pyas" in r["Name"]:
            print("   %-75s calls=%s avg_us=%.1f" % (r["Name"][:75], r["Calls"], float(r["AverageNs"]) / 1e3))
