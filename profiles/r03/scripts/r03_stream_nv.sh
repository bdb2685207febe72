# k_axes_col_stream items per lane (NV) and ring depth variants: parity + per-chunk axes sweep
set -o pipefail
mkdir -p gpurun_out/r03
V=$PWD/pyactivestorage_amd/lib/variants
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_axes_stream.py > gpurun_out/r03/nv_tests_default.log 2>&1 || exit 1
for v in nv2 nv2d1; do
  PYAS_LIB=$V/libpyas_$v.so timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_axes_stream.py > gpurun_out/r03/nv_tests_$v.log 2>&1 || exit 1
done
for rep in 1 2; do
for v in default nv2 nv2d1; do
  if [ $v = default ]; then lib=""; else lib=$V/libpyas_$v.so; fi
  for c in 0 8 32; do
    PYAS_LIB=$lib PYAS_COL_STREAM=$c timeout -k 10 120 python -u tools/bench_axes.py > gpurun_out/r03/nv_${v}_plain_${c}_$rep.json 2>&1 || exit 1
    PYAS_LIB=$lib PYAS_COL_STREAM=$c timeout -k 10 120 python -u tools/bench_axes.py --shuffle > gpurun_out/r03/nv_${v}_shuf_${c}_$rep.json 2>&1 || exit 1
  done
done
done
