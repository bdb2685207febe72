set -o pipefail
mkdir -p gpurun_out/r03
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_inflate.py tests/test_gpu_coalesced.py tests/test_gpu_golden.py > gpurun_out/r03/zlib_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_dropin.py --zlib --chunks 2048 --trials 3 > gpurun_out/r03/dropin_zlib_host.json 2> gpurun_out/r03/dropin_zlib_host.err || exit 1
timeout -k 10 300 env PYAS_COALESCE_INFLATE=device PYAS_PERCALL_INFLATE=device python -u tools/bench_dropin.py --zlib --chunks 2048 --trials 3 > gpurun_out/r03/dropin_zlib_device.json 2> gpurun_out/r03/dropin_zlib_device.err || exit 1
