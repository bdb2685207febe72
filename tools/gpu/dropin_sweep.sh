set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -s tests/test_gpu_coalesced.py tests/test_gpu_resident.py > gpurun_out/r02/test_coalesced.log 2>&1 || exit 2
PYAS_COALESCE_COPY=caller PYAS_COALESCE_SYNC=spin timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -s tests/test_gpu_coalesced.py >> gpurun_out/r02/test_coalesced.log 2>&1 || exit 3
timeout -k 10 300 python -u tools/bench_dropin.py --chunks 8192 --ceiling-read > gpurun_out/r02/dropin_bench.json 2> gpurun_out/r02/dropin_bench.err || exit 4
