# k_axes_col_stream: parity tests, then per-chunk axes sweep over chunks per workgroup
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_axes_stream.py tests/test_gpu_axes_dense.py tests/test_gpu_axes_fold.py > gpurun_out/r03/stream_tests.log 2>&1 || exit 1
for c in 0 2 4 8 16 32; do
  PYAS_COL_STREAM=$c timeout -k 10 120 python -u tools/bench_axes.py > gpurun_out/r03/stream_plain_$c.json 2>&1 || exit 1
  PYAS_COL_STREAM=$c timeout -k 10 120 python -u tools/bench_axes.py --shuffle > gpurun_out/r03/stream_shuf_$c.json 2>&1 || exit 1
done
timeout -k 10 120 python -u tools/bench_axes.py --fold > gpurun_out/r03/fold_plain.json 2>&1 || exit 1
timeout -k 10 120 python -u tools/bench_axes.py --fold --shuffle > gpurun_out/r03/fold_shuf.json 2>&1 || exit 1
