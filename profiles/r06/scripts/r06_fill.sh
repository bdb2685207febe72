# round 6: k_reduce_axes 16-B column split rules (PYAS_AXES_FILL 0/1/2) on the strided
# partial-axis query and the cut-chunk generic shapes; axes tests under the fill rule
set -o pipefail
O=gpurun_out/r06/fill
R=$GRAFT_REPO_ROOT
mkdir -p $O
PYAS_AXES_FILL=2 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "axes or active or records or zero_sign" > $O/gpu_tests_fill2.log 2>&1 || exit 1
for f in 0 1 2; do
  PYAS_AXES_FILL=$f bash $R/tools/profile_query.sh c3_stride 3 r06fill$f || exit 1
done
