# one tile per wave by default in the LDS row layout: parity + per-chunk axes, two repeats
set -o pipefail
O=gpurun_out/r03/tpw1
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_axes_rowlds.py tests/test_gpu_axes_dense.py > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 120 python -u tools/bench_axes.py > $O/plain_$r.json 2>&1 || exit 1
  timeout -k 10 120 python -u tools/bench_axes.py --shuffle > $O/shuf_$r.json 2>&1 || exit 1
done
