# inflate variants: timing + phase profile per variant library
set -o pipefail
mkdir -p gpurun_out/r02i
for v in $INFL_VARIANTS; do
  PYAS_LIB=pyactivestorage_amd/lib/libpyas_hip_$v.so timeout -k 10 200 python -u tools/bench_inflate.py --chunks 2048 --sweep 32 --cpu-threads 1 > gpurun_out/r02i/bench_$v.json 2> gpurun_out/r02i/bench_$v.err || exit 2
done
for v in $INFL_PROF; do
  PYAS_LIB=pyactivestorage_amd/lib/libpyas_hip_$v.so timeout -k 10 120 python -u tools/bench_inflate.py --chunks 32 --reps 1 --cpu-threads 1 > gpurun_out/r02i/prof_$v.txt 2>&1 || exit 3
done
