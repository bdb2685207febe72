"""Summarise rocprofv3 output of tools/query_c3.py runs (one query shape):
per pyas kernel the average duration (--kernel-trace --stats) and the HBM
bytes per dispatch from separate --pmc FETCH_SIZE / WRITE_SIZE passes
(MI355X_MICROARCH.md: FETCH_SIZE x 1024 x 2 for 16-B streaming reads,
WRITE_SIZE x 1024 exact for 16-B stores), beside the query's selected and
touched-line bytes (bench.selected_and_touched).

    python tools/query_summary.py NAME IDX STATS.csv FETCH.csv WRITE.csv QUERY.json OUT.json
"""
import csv
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import bench  # noqa: E402


def stats(path):
    out = {}
    for r in csv.DictReader(open(path)):
        if "pyas::" in r["Name"]:
            out[r["Name"]] = {"calls": int(r["Calls"]), "avg_us": round(float(r["AverageNs"]) / 1e3, 2)}
    return out


def pmc(path, counter):
    per = {}
    for r in csv.DictReader(open(path)):
        if "pyas::" in r["Kernel_Name"] and r["Counter_Name"] == counter:
            per.setdefault(r["Kernel_Name"], []).append(float(r["Counter_Value"]))
    return {k: sum(v) / len(v) for k, v in per.items()}


def main():
    name, idx, st, fe, wr, qj, out = sys.argv[1:8]
    label, mk, axis, method = bench.ACTIVE_EXTRAS[name][int(idx)]
    sel, touched = bench.selected_and_touched(mk(), bench.CONFIGS["c3"]["shape"], bench.CONFIGS["c3"]["chunks"], 4)
    ks = stats(st)
    f = pmc(fe, "FETCH_SIZE")
    w = pmc(wr, "WRITE_SIZE")
    for k, v in ks.items():
        if k in f:
            v["fetch_bytes"] = int(f[k] * 1024 * 2)
        if k in w:
            v["write_bytes"] = int(w[k] * 1024)
    kern_us = sum(v["avg_us"] * v["calls"] for v in ks.values()) / max(1, max(v["calls"] for v in ks.values()))
    q = [json.loads(x) for x in open(qj) if x.startswith("{")]
    main_k = max(ks, key=lambda k: ks[k]["avg_us"])
    mk_ = ks[main_k]
    rep = {"query": label, "axis": axis, "method": method, "selected_bytes": sel, "touched_line_bytes": touched,
           "end_to_end": q[-1] if q else None, "kernels": ks, "dominant_kernel": main_k,
           "dominant_frac_selected": round(sel / (mk_["avg_us"] * 1e-6) / 8e12, 4),
           "dominant_frac_touched": round(touched / (mk_["avg_us"] * 1e-6) / 8e12, 4),
           "dominant_fetch_over_touched": round(mk_.get("fetch_bytes", 0) / touched, 4) if touched else None,
           "pyas_kernel_us_per_query": round(kern_us, 1),
           "note": "fractions of 8 TB/s; fetch = FETCH_SIZE x 2 (gfx950 16-B read correction)"}
    json.dump(rep, open(out, "w"), indent=1)
    print(json.dumps({k: rep[k] for k in ("query", "axis", "method", "dominant_kernel", "dominant_frac_selected",
                                           "dominant_frac_touched", "dominant_fetch_over_touched")}))


if __name__ == "__main__":
    main()
