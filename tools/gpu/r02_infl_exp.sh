# inflate variants: parity of each variant library, then timing
set -o pipefail
mkdir -p gpurun_out/r02i
for v in $INFL_VARIANTS; do
  PYAS_LIB=pyactivestorage_amd/lib/libpyas_hip_$v.so timeout -k 10 200 python -u -m pytest -x -q --timeout 60 --timeout-method thread tests/test_gpu_inflate.py > gpurun_out/r02i/tests_$v.log 2>&1 || exit 1
  PYAS_LIB=pyactivestorage_amd/lib/libpyas_hip_$v.so timeout -k 10 200 python -u tools/bench_inflate.py --chunks 2048 --reps 5 --sweep 32 --cpu-threads 1 > gpurun_out/r02i/exp_$v.json 2> gpurun_out/r02i/exp_$v.err || exit 2
done
