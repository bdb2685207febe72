# Active zlib full mean by inflate group count (contiguous staging)
set -o pipefail
mkdir -p gpurun_out/r02s
for g in 2 3 4 6; do
  PYAS_INFLATE_GROUPS=$g timeout -k 10 300 python -u tools/bench_active.py --zlib --axes none --reps 5 > gpurun_out/r02s/zlib_g$g.json 2> gpurun_out/r02s/zlib_g$g.err || exit 2
done
