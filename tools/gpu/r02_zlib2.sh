# Active zlib: contiguous compressed staging (one H2D per slot): parity + query time
set -o pipefail
mkdir -p gpurun_out/r02s
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_active_files.py tests/test_gpu_resident.py tests/test_gpu_active.py tests/test_gpu_distributed_active.py > gpurun_out/r02s/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_active.py --zlib --reps 3 > gpurun_out/r02s/zlib_contig.json 2> gpurun_out/r02s/zlib_contig.err || exit 2
