# round 5: span walk per lane group (U=2) -- parity, split probe, query profiles
set -o pipefail
O=gpurun_out/r05/q4
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_spans.py tests/test_gpu_reduce_chunk.py tests/test_gpu_axes_cuts.py tests/test_gpu_axes_dense.py tests/test_gpu_axes_rowlds.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe_reduce_sel.py > $O/probe_sel.json 2>&1 || exit 1
PYAS_SPANS=2 timeout -k 10 300 python -u tools/probe_reduce_sel.py > $O/probe_sel_spans2.json 2>&1 || exit 1
for q in "c3_slab 0" "c3_slab 4" "c3_slab 5" "c3_stride 0" "c3_stride 1" "c3_stride 2"; do
  bash tools/profile_query.sh $q r05 >> $O/qprof.log 2>&1 || exit 1
done
