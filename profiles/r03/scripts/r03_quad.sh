# quad-cooperative shuffled plane loads in k_axes_col_stream: parity, then shuffled per-chunk sweep vs the ldv build
set -o pipefail
O=gpurun_out/r03/quad
mkdir -p $O
V=$PWD/pyactivestorage_amd/lib/variants
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_axes_stream.py tests/test_gpu_axes_dense.py > $O/tests.log 2>&1 || exit 1
B="timeout -k 10 120 python -u tools/bench_axes.py --shuffle"
for rep in 1 2; do
  PYAS_COL_STREAM=0 $B > $O/off_$rep.json 2>&1 || exit 1
  for c in 8 16 32; do
    PYAS_COL_STREAM=$c $B > $O/quad_${c}_$rep.json 2>&1 || exit 1
    PYAS_LIB=$V/libpyas_noquad.so PYAS_COL_STREAM=$c $B > $O/noquad_${c}_$rep.json 2>&1 || exit 1
  done
done
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_axes_fold.py > $O/tests_fold.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 120 python -u tools/bench_axes.py --fold --shuffle > $O/fold_quad_$rep.json 2>&1 || exit 1
  PYAS_LIB=$V/libpyas_noquad.so timeout -k 10 120 python -u tools/bench_axes.py --fold --shuffle > $O/fold_noquad_$rep.json 2>&1 || exit 1
done
