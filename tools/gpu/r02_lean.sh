# lean column fold: parity (fold tests), then C3 fold throughput: auto (split), unsplit, k_axes_fold
set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_axes_fold.py > gpurun_out/r02/lean_tests.log 2>&1 || exit 1
for lean in auto 1 0; do
  for mode in "--fold" "--fold --shuffle"; do
    if [ $lean = auto ]; then unset PYAS_FOLD_LEAN; else export PYAS_FOLD_LEAN=$lean; fi
    timeout -k 10 120 python -u tools/bench_axes.py $mode | sed "s/^/lean=$lean /" >> gpurun_out/r02/lean_bench.txt 2>> gpurun_out/r02/lean_bench.err || exit 2
  done
done
