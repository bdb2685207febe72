# pinned result arrays: tests, then resident queries and method=None selects A/B (pool vs pageable)
set -o pipefail
mkdir -p gpurun_out/r02e
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_result_pool.py tests/test_gpu_resident.py tests/test_gpu_active.py tests/test_gpu_active_select.py tests/test_gpu_active_files.py tests/test_gpu_format.py > gpurun_out/r02e/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u tools/bench_active.py --resident --reps 30 | tail -n 1 | sed "s/^/pinned /" >> gpurun_out/r02e/resident_ab.txt 2>> gpurun_out/r02e/resident.err || exit 2
  PYAS_RESULT_PINNED_MIB=0 timeout -k 10 300 python -u tools/bench_active.py --resident --reps 30 | tail -n 1 | sed "s/^/pageable /" >> gpurun_out/r02e/resident_ab.txt 2>> gpurun_out/r02e/resident.err || exit 3
done
PYAS_RESULT_PINNED_MIB=2048 timeout -k 10 300 python -u tools/probe_select.py | sed "s/^/pinned /" >> gpurun_out/r02e/select_ab.txt 2>> gpurun_out/r02e/select.err || exit 4
PYAS_RESULT_PINNED_MIB=0 timeout -k 10 300 python -u tools/probe_select.py | sed "s/^/pageable /" >> gpurun_out/r02e/select_ab.txt 2>> gpurun_out/r02e/select.err || exit 5
