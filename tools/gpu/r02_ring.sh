# ring column walk in the per-chunk dense kernel: parity, then C3 per-chunk axes (plain, shuffled) and folds
set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_axes_dense.py tests/test_gpu_axes_fold.py tests/test_gpu_reduce_chunk.py tests/test_gpu_mask_trim.py > gpurun_out/r02/ring_tests.log 2>&1 || exit 1
for mode in "" "--shuffle" "--fold" "--fold --shuffle"; do
  timeout -k 10 120 python -u tools/bench_axes.py $mode >> gpurun_out/r02/ring_bench.jsonl 2>> gpurun_out/r02/ring_bench.err || exit 2
done
