# round 6: the strided column walk (k_reduce_axes col_vec: per-chunk split, 8 rows in flight,
# grouped sums): axes/active GPU tests, then rocprof of the c3_stride queries
set -o pipefail
O=gpurun_out/r06/stride
R=$GRAFT_REPO_ROOT
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "axes or active or golden or records or spans or zero_sign" > $O/gpu_tests.log 2>&1 || exit 1
for q in "c3_stride 3" "c3_stride 0" "c3_stride 4"; do
  bash $R/tools/profile_query.sh $q r06 || exit 1
done
