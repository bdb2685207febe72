set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 400 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_resident.py tests/test_gpu_active.py tests/test_gpu_active_files.py tests/test_gpu_active_select.py tests/test_gpu_distributed_active.py > gpurun_out/r02/resident_tests.log 2>&1 || exit 1
timeout -k 10 400 python -u tools/bench_active.py --resident --reps 20 --profile > gpurun_out/r02/active_resident_prof.log 2>&1 || exit 2
