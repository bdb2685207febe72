# closing: full GPU suite + smoke with the final tree
set -o pipefail
mkdir -p gpurun_out/r02c2
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02c2/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02c2/smoke.log 2>&1 || exit 2
