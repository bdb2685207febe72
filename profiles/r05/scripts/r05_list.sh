# round 5: index lists as the last span dim read from an LDS copy -- parity of
# the selection tests, then the stride/list query shapes (rocprof + FETCH)
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/list
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_spans.py tests/test_gpu_golden.py tests/test_gpu_active.py tests/test_gpu_reduce_chunk.py tests/test_gpu_active_select.py > $O/tests.log 2>&1 || exit 1
for q in "c3_stride 2" "c3_stride 0" "c3_stride 1" "c3_slab 0"; do
  bash $R/tools/profile_query.sh $q r05b || exit 1
done
