# after the last library change: combine/fold/chained parity, smoke, default bench
set -o pipefail
mkdir -p gpurun_out/r02f2
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_axes_fold.py tests/test_gpu_chained.py tests/test_gpu_active.py tests/test_gpu_resident.py tests/test_gpu_golden.py > gpurun_out/r02f2/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02f2/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > gpurun_out/r02f2/bench_default.json 2> gpurun_out/r02f2/bench_default.err || exit 3
