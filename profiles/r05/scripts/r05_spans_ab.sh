# round 5: PYAS_SPANS 0 / 1 / 2 on C5 and the C3 query shapes (same box)
set -o pipefail
O=gpurun_out/r05/spans_ab
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_spans.py tests/test_gpu_axes_slab.py > $O/tests.log 2>&1 || exit 1
for sp in 1 2 0; do
  PYAS_SPANS=$sp timeout -k 10 400 python -u bench.py --steps 10 --extra c5,c3_slab,c3_stride --extra-steps 10 --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 > $O/bench_spans$sp.json 2> $O/bench_spans$sp.err || exit 1
done
