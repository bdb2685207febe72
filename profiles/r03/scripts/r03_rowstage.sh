# staged LDS-row partial stores: parity, per-chunk axes A/B is against the previous run's numbers on the same script
set -o pipefail
O=gpurun_out/r03/rowstage
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_axes_rowlds.py tests/test_gpu_axes_dense.py tests/test_gpu_axes_stream.py tests/test_gpu_axes_fold.py > $O/tests.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 120 python -u tools/bench_axes.py > $O/pc_plain_$rep.json 2>&1 || exit 1
  timeout -k 10 120 python -u tools/bench_axes.py --shuffle > $O/pc_shuffle_$rep.json 2>&1 || exit 1
done
