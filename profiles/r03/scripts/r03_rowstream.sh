# k_axes_lds_stream: parity, then per-chunk (2,) sweep over chunks per workgroup and tiles per wave
set -o pipefail
O=gpurun_out/r03/rs
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_axes_stream.py tests/test_gpu_axes_rowlds.py > $O/tests.log 2>&1 || exit 1
B="timeout -k 10 120 python -u tools/bench_axes.py"
for k in "" "--shuffle"; do
  tag=${k:-plain}; tag=${tag#--}
  PYAS_ROW_STREAM=0 $B $k > $O/rs_0_2_${tag}.json 2>&1 || exit 1
  for c in 4 16 64; do for t in 1 2 8; do
    PYAS_ROW_STREAM=$c PYAS_ROW_STREAM_TPW=$t $B $k > $O/rs_${c}_${t}_${tag}.json 2>&1 || exit 1
  done; done
  PYAS_ROW_STREAM=0 $B $k > $O/rs_0_2_${tag}_b.json 2>&1 || exit 1
done
