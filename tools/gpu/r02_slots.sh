# ingest slot geometry vs Active file queries (zlib and uncompressed)
set -o pipefail
mkdir -p gpurun_out/r02s
for sl in 16x64 64x16 32x32 128x8; do
  PYAS_INGEST_SLOTS=$sl timeout -k 10 300 python -u tools/bench_active.py --zlib --axes none --reps 3 > gpurun_out/r02s/zlib_$sl.json 2> gpurun_out/r02s/zlib_$sl.err || exit 1
  PYAS_INGEST_SLOTS=$sl timeout -k 10 300 python -u tools/bench_active.py --axes none --reps 3 > gpurun_out/r02s/plain_$sl.json 2> gpurun_out/r02s/plain_$sl.err || exit 2
done
