# lean fold: repeated A/B (split auto vs unsplit), then rocprofv3 kernel stats + FETCH_SIZE of the fold and per-chunk axes benches
set -o pipefail
mkdir -p gpurun_out/r02/prof
export TMPDIR=/tmp
for rep in 1 2 3; do
  for lean in auto 1; do
    if [ $lean = auto ]; then unset PYAS_FOLD_LEAN; else export PYAS_FOLD_LEAN=$lean; fi
    timeout -k 10 120 python -u tools/bench_axes.py --fold | sed "s/^/lean=$lean /" >> gpurun_out/r02/lean_ab.txt 2>> gpurun_out/r02/lean_ab.err || exit 1
  done
done
unset PYAS_FOLD_LEAN
for mode in fold foldshuffle plain shuffle; do
  case $mode in fold) a="--fold";; foldshuffle) a="--fold --shuffle";; plain) a="";; shuffle) a="--shuffle";; esac
  rm -rf /tmp/pt_$mode /tmp/pf_$mode
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/pt_$mode -o run -- python3 tools/bench_axes.py $a > gpurun_out/r02/prof/${mode}_trace.log 2>&1 || exit 2
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pf_$mode -o run -- python3 tools/bench_axes.py $a > gpurun_out/r02/prof/${mode}_fetch.log 2>&1 || exit 3
  cp $(find /tmp/pt_$mode -name '*kernel_stats.csv' | head -n 1) gpurun_out/r02/prof/axes_${mode}_kernel_stats.csv
  cp $(find /tmp/pf_$mode -name '*counter_collection.csv' | head -n 1) gpurun_out/r02/prof/axes_${mode}_pmc_fetch_size.csv
done
