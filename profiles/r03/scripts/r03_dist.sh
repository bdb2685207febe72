set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_bench_dist.py "tests/test_gpu_fullsize.py::test_full_size_samples_against_oracle" tests/test_gpu_coalesced.py -s > gpurun_out/r03/dist_oracle_tests.log 2>&1 || exit 1
