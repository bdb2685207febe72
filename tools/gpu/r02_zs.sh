set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 600 python -u -m pytest -x -q -s --timeout 300 --timeout-method thread tests/test_gpu_zero_sign.py tests/test_gpu_golden.py tests/test_gpu_coalesced.py tests/test_gpu_active.py tests/test_gpu_resident.py > gpurun_out/r02/zs_tests.log 2>&1 || exit 1
