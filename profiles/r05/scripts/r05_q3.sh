# round 5: cut map by ballot, one generic block per chunk; k_reduce_u split probe
set -o pipefail
O=gpurun_out/r05/q3
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_axes_cuts.py tests/test_gpu_axes_dense.py tests/test_gpu_resident.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/probe_reduce_sel.py > $O/probe_sel.json 2>&1 || exit 1
PYAS_SPANS=2 timeout -k 10 300 python -u tools/probe_reduce_sel.py > $O/probe_sel_spans2.json 2>&1 || exit 1
for q in "c3_slab 4" "c3_slab 5"; do
  bash tools/profile_query.sh $q r05 >> $O/qprof.log 2>&1 || exit 1
done
