# full GPU test suite + default bench on the current tree (one box call)
set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r03/gpu_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r03/bench_full.json 2> gpurun_out/r03/bench_full.err || exit 1
