# pipelined coalescer: parity + drop-in rate by depth; fold-kernel tuning variants
set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_coalesced.py tests/test_gpu_golden.py > gpurun_out/r02/coalesced_tests.log 2>&1 || exit 1
for d in 1 2 4 8; do
  PYAS_COALESCE_DEPTH=$d timeout -k 10 120 python -u tools/bench_dropin.py --chunks 2048 --gpu-only --trials 3 --ceiling-read >> gpurun_out/r02/dropin_depth.jsonl 2>> gpurun_out/r02/dropin_depth.err || exit 2
done
for v in w4 w5 u4 u4w5; do
  PYAS_LIB=$PWD/pyactivestorage_amd/lib/variants/libpyas_$v.so timeout -k 10 120 python -u tools/bench_axes.py --fold > gpurun_out/r02/fold_$v.json 2>> gpurun_out/r02/fold_var.err || exit 3
  PYAS_LIB=$PWD/pyactivestorage_amd/lib/variants/libpyas_$v.so timeout -k 10 120 python -u tools/bench_axes.py > gpurun_out/r02/axes_$v.json 2>> gpurun_out/r02/fold_var.err || exit 4
done
