# CU-scaled stream targets: parity (stream + auto size test) and per-chunk axes, two repeats
set -o pipefail
O=gpurun_out/r03/cpb2
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_axes_stream.py tests/test_gpu_coalesced.py > $O/tests.log 2>&1 || exit 1
for r in 1 2; do
  timeout -k 10 120 python -u tools/bench_axes.py > $O/plain_$r.json 2>&1 || exit 1
  timeout -k 10 120 python -u tools/bench_axes.py --shuffle > $O/shuf_$r.json 2>&1 || exit 1
done
