# shuffled chunks on the dense partial-axis kernels: parity, then C3 throughput
set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_axes_dense.py tests/test_gpu_axes_fold.py tests/test_gpu_axes_rowlds.py > gpurun_out/r02/axes_tests.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/bench_axes.py --shuffle > gpurun_out/r02/axes_bench_shuffled.json 2> gpurun_out/r02/axes_bench.err || exit 2
timeout -k 10 120 python -u tools/bench_axes.py > gpurun_out/r02/axes_bench_dense.json 2>> gpurun_out/r02/axes_bench.err || exit 3
