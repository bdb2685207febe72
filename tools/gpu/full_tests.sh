# full GPU test suite + drop-in bench (one box call)
set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_dropin.py --chunks 8192 > gpurun_out/r02/dropin_bench.json 2> gpurun_out/r02/dropin_bench.err || exit 2
