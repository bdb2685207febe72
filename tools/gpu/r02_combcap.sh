# wave combine bounded to <= 2^17 outputs: fold/combine parity + resident box queries
set -o pipefail
mkdir -p gpurun_out/r02x
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_axes_fold.py tests/test_gpu_resident.py tests/test_gpu_active.py tests/test_gpu_distributed_active.py tests/test_gpu_result_pool.py > gpurun_out/r02x/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_active.py --resident --reps 30 > gpurun_out/r02x/resident.json 2> gpurun_out/r02x/resident.err || exit 2
