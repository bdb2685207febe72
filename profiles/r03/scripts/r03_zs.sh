set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 900 python -u -m pytest -x -v --timeout 300 --timeout-method thread tests/test_gpu_zero_sign.py tests/test_gpu_golden.py tests/test_gpu_coalesced.py tests/test_gpu_distributed_active.py -s > gpurun_out/r03/zs_tests.log 2>&1 || exit 1
