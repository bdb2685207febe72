set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_fullsize.py -k oracle tests/test_gpu_bench_dist.py -s > gpurun_out/r03/dist_oracle_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > gpurun_out/r03/bench_default.json 2> gpurun_out/r03/bench_default.err || exit 1
