# round 4 rocprofv3 evidence, C3 partial axes (one axis set per run): kernel
# trace + stats, then FETCH_SIZE and WRITE_SIZE passes (separate runs, no
# traces); per-chunk kernels with compact sum records, and the zero-heavy
# zero-sign kernels (FETCH_SIZE); then the full per-chunk sweep (the grid
# rule re-measure) in both partial forms.
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r04/axprof
mkdir -p $O
cd /tmp
summ() {
python3 - "$@" <<'PY'
import csv, sys
rows = {}
for f in sys.argv[1:]:
    for r in csv.DictReader(open(f)):
        if "pyas" not in r["Kernel_Name"]:
            continue
        k = (r["Kernel_Name"].split("(")[0], r["Counter_Name"])
        rows.setdefault(k, []).append(float(r["Counter_Value"]))
print("kernel,counter,dispatches,avg_per_dispatch")
for (k, c), v in sorted(rows.items()):
    print(f'"{k}",{c},{len(v)},{sum(v) / len(v):.1f}')
PY
}
for spec in "plainrec:0" "plainrec:1" "plainrec:2" "shufrec:0" "shufrec:1" "shufrec:2" "shuf:1"; do
  kind=${spec%%:*}; ax=${spec#*:}
  case $kind in plainrec) a="--rec sum";; shufrec) a="--shuffle --rec sum";; shuf) a="--shuffle";; esac
  tag=${kind}_$ax
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ap/$tag/trace -o run -- python3 $R/tools/bench_axes.py $a --only $ax > $O/${tag}_trace.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/ap/$tag/fetch -o run -- python3 $R/tools/bench_axes.py $a --only $ax > $O/${tag}_fetch.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/ap/$tag/write -o run -- python3 $R/tools/bench_axes.py $a --only $ax > $O/${tag}_write.log 2>&1 || exit 1
  cp $(find /tmp/ap/$tag/trace -name '*kernel_stats.csv' | head -n 1) $O/${tag}_kernel_stats.csv
  summ "$(find /tmp/ap/$tag/fetch -name '*counter_collection.csv' | head -n 1)" "$(find /tmp/ap/$tag/write -name '*counter_collection.csv' | head -n 1)" > $O/${tag}_pmc.csv || exit 1
done
# zero-heavy zero-sign kernels: FETCH_SIZE of k_tie_pick / k_tie_scan / k_tie_grid / the ZS folds
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/ap/zeros/fetch -o run -- python3 $R/tools/bench_zeros.py --zeros 0.5 --axes none,0,2 --reps 2 > $O/zeros50_fetch.log 2>&1 || exit 1
summ "$(find /tmp/ap/zeros/fetch -name '*counter_collection.csv' | head -n 1)" > $O/zeros50_pmc.csv || exit 1
cd $R
for a in "" "--rec sum" "--shuffle" "--shuffle --rec sum" "--fold" "--fold --shuffle"; do
  timeout -k 10 300 python3 -u tools/bench_axes.py $a >> $O/sweep.jsonl 2>> $O/sweep.err || exit 1
done
