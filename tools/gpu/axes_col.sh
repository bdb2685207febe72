# partial-axis kernels: parity, then per-chunk and folded throughput, plain and shuffled
set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_mask_trim.py tests/test_gpu_axes_dense.py tests/test_gpu_axes_fold.py tests/test_gpu_axes_rowlds.py tests/test_gpu_reduce_chunk.py tests/test_gpu_active.py tests/test_gpu_resident.py tests/test_gpu_chained.py > gpurun_out/r02/axes_tests.log 2>&1 || exit 1
for v in "" "--shuffle" "--fold" "--fold --shuffle"; do
  timeout -k 10 120 python -u tools/bench_axes.py $v >> gpurun_out/r02/axes_bench.jsonl 2>> gpurun_out/r02/axes_bench.err || exit 2
done
timeout -k 10 300 python bench.py --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 > gpurun_out/r02/bench_quick.json 2> gpurun_out/r02/bench_quick.err || exit 3
