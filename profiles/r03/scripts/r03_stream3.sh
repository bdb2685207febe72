# k_axes_col_stream with per-geometry items per lane: parity, then per-chunk axes (auto vs off) and fold
set -o pipefail
O=gpurun_out/r03/s3
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_axes_stream.py tests/test_gpu_axes_dense.py tests/test_gpu_axes_fold.py tests/test_gpu_coalesced.py tests/test_gpu_reduce_chunk.py > $O/tests.log 2>&1 || exit 1
B="timeout -k 10 120 python -u tools/bench_axes.py"
for rep in 1 2; do
  for k in "" "--shuffle"; do
    tag=${k:-plain}; tag=${tag#--}
    PYAS_COL_STREAM=0 $B $k > $O/pc_off_${tag}_$rep.json 2>&1 || exit 1
    $B $k > $O/pc_auto_${tag}_$rep.json 2>&1 || exit 1
  done
done
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
