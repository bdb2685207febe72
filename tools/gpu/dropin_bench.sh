set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 300 python -u tools/bench_dropin.py --ceiling-read > gpurun_out/r02/dropin_bench_default.json 2> gpurun_out/r02/dropin_bench.err || exit 1
timeout -k 10 300 python -u tools/bench_dropin.py --chunks 8192 --ceiling-read > gpurun_out/r02/dropin_bench_8192.json 2>> gpurun_out/r02/dropin_bench.err || exit 2
timeout -k 10 300 python -u tools/bench_dropin.py --zlib --chunks 1024 --percall-chunks 256 > gpurun_out/r02/dropin_bench_zlib.json 2>> gpurun_out/r02/dropin_bench.err || exit 3
