set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 300 python -u bench.py > gpurun_out/r03/bench_baseline.json 2> gpurun_out/r03/bench_baseline.err || exit 1
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_golden.py tests/test_gpu_zero_sign.py > gpurun_out/r03/golden.log 2>&1 || exit 1
