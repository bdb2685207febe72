# round 6: the strided column walk with 16 rows in flight per lane (was 8): axes tests, rocprof
set -o pipefail
O=gpurun_out/r06/u16
R=$GRAFT_REPO_ROOT
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "axes or active or records or zero_sign or golden" > $O/gpu_tests.log 2>&1 || exit 1
for q in "c3_stride 3"; do
  bash $R/tools/profile_query.sh $q r06u16 || exit 1
done
