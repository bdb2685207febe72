# stream NV=2/4 and lean-fold NV=2 variants: parity with each, then per-chunk and fold axes sweeps
set -o pipefail
mkdir -p gpurun_out/r03/s2
O=gpurun_out/r03/s2
V=$PWD/pyactivestorage_amd/lib/variants
T="timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread"
$T tests/test_gpu_axes_stream.py tests/test_gpu_axes_fold.py > $O/tests_default.log 2>&1 || exit 1
for v in nv4d1 nv2d1; do PYAS_LIB=$V/libpyas_$v.so $T tests/test_gpu_axes_stream.py > $O/tests_$v.log 2>&1 || exit 1; done
for v in lean2 lean2d1; do PYAS_LIB=$V/libpyas_$v.so $T tests/test_gpu_axes_fold.py > $O/tests_$v.log 2>&1 || exit 1; done
B="timeout -k 10 120 python -u tools/bench_axes.py"
for rep in 1 2; do
  for k in "" "--shuffle"; do
    tag=${k:-plain}; tag=${tag#--}
    PYAS_COL_STREAM=0 $B $k > $O/pc_default_0_${tag}_$rep.json 2>&1 || exit 1
    PYAS_COL_STREAM=32 $B $k > $O/pc_default_32_${tag}_$rep.json 2>&1 || exit 1
    for c in 16 32; do PYAS_LIB=$V/libpyas_nv2d1.so PYAS_COL_STREAM=$c $B $k > $O/pc_nv2d1_${c}_${tag}_$rep.json 2>&1 || exit 1; done
    for c in 4 8 16; do PYAS_LIB=$V/libpyas_nv4d1.so PYAS_COL_STREAM=$c $B $k > $O/pc_nv4d1_${c}_${tag}_$rep.json 2>&1 || exit 1; done
    $B --fold $k > $O/fold_default_${tag}_$rep.json 2>&1 || exit 1
    for v in lean2 lean2d1; do PYAS_LIB=$V/libpyas_$v.so $B --fold $k > $O/fold_${v}_${tag}_$rep.json 2>&1 || exit 1; done
  done
done
