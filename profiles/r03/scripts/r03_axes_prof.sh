# rocprofv3 evidence for the partial-axis kernels on C3, one axis set per run:
# kernel trace + stats, then FETCH_SIZE and WRITE_SIZE passes (separate runs, no traces)
set -o pipefail
export TMPDIR=/tmp
R=$PWD
O=$R/gpurun_out/r03/axprof
mkdir -p $O
cd /tmp
for spec in "plain:0" "plain:1" "plain:2" "shuffle:0" "shuffle:1" "shuffle:2" "fold:0" "fold:1" "foldshuffle:0" "foldshuffle:1"; do
  kind=${spec%%:*}; ax=${spec#*:}
  case $kind in plain) a="";; shuffle) a="--shuffle";; fold) a="--fold";; foldshuffle) a="--fold --shuffle";; esac
  tag=${kind}_$ax
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ap/$tag/trace -o run -- python3 $R/tools/bench_axes.py $a --only $ax > $O/${tag}_trace.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/ap/$tag/fetch -o run -- python3 $R/tools/bench_axes.py $a --only $ax > $O/${tag}_fetch.log 2>&1 || exit 1
  timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d /tmp/ap/$tag/write -o run -- python3 $R/tools/bench_axes.py $a --only $ax > $O/${tag}_write.log 2>&1 || exit 1
  cp $(find /tmp/ap/$tag/trace -name '*kernel_stats.csv' | head -n 1) $O/${tag}_kernel_stats.csv
  python3 - "$(find /tmp/ap/$tag/fetch -name '*counter_collection.csv' | head -n 1)" "$(find /tmp/ap/$tag/write -name '*counter_collection.csv' | head -n 1)" > $O/${tag}_pmc.csv <<'PY' || exit 1
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
done
