set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread -s tests/test_gpu_coalesced.py > gpurun_out/r02/test_coalesced.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_dropin.py --chunks 4096 > gpurun_out/r02/dropin_bench.json 2> gpurun_out/r02/dropin_bench.err || exit 2
timeout -k 10 300 python -u tools/bench_dropin.py --chunks 4096 --zlib > gpurun_out/r02/dropin_bench_zlib.json 2> gpurun_out/r02/dropin_bench_zlib.err || exit 3
