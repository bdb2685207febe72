set -o pipefail
mkdir -p gpurun_out/r02i
for w in 13 14 15; do
  timeout -k 10 200 python -u tools/bench_inflate.py --chunks 2048 --wbits $w --sweep 32,1024 --cpu-threads 1 > gpurun_out/r02i/wbits_$w.json 2> gpurun_out/r02i/wbits_$w.err || exit 2
done
PYAS_LIB=pyactivestorage_amd/lib/libpyas_hip_prof0.so timeout -k 10 120 python -u tools/bench_inflate.py --chunks 32 --reps 1 --cpu-threads 1 --wbits 14 > gpurun_out/r02i/prof_w14.txt 2>&1 || exit 3
