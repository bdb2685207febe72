# whole/boundary split launch: parity (chained, golden, hyperslab paths), then C5 with and without the split
set -o pipefail
mkdir -p gpurun_out/r02s
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_chained.py tests/test_gpu_golden.py tests/test_gpu_reduce_chunk.py tests/test_gpu_active.py tests/test_gpu_active_select.py tests/test_gpu_resident.py tests/test_gpu_distributed_active.py tests/test_gpu_zero_sign.py > gpurun_out/r02s/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u bench.py --config c5 --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 --extra none > gpurun_out/r02s/c5_split.json 2> gpurun_out/r02s/c5.err || exit 2
PYAS_SPLIT_WHOLE=0 timeout -k 10 300 python -u bench.py --config c5 --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 --extra none > gpurun_out/r02s/c5_one.json 2>> gpurun_out/r02s/c5.err || exit 3
timeout -k 10 300 python -u bench.py --config c5 --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 --extra none > gpurun_out/r02s/c5_split2.json 2>> gpurun_out/r02s/c5.err || exit 4
