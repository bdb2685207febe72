# r02 re-entry: full GPU suite, smoke, default bench (one box call)
set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r02/smoke.log 2>&1 || exit 2
timeout -k 10 400 python bench.py > gpurun_out/r02/bench_default.json 2> gpurun_out/r02/bench_default.err || exit 3
