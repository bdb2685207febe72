# drop-in reduce_chunk from a 30-thread pool: uncompressed and shuffle+zlib, this round's library
set -o pipefail
O=gpurun_out/r03/dropin
mkdir -p $O
timeout -k 10 300 python -u tools/bench_dropin.py --chunks 8192 > $O/plain.json 2> $O/plain.err || exit 1
timeout -k 10 300 python -u tools/bench_dropin.py --zlib --chunks 2048 --trials 3 > $O/zlib.json 2> $O/zlib.err || exit 1
timeout -k 10 300 python -u tools/bench_axes.py --only 2 > $O/axes2.json 2>&1 || exit 1
