# round 6: the remaining bench query shapes under rocprof on the final binary
set -o pipefail
R=$GRAFT_REPO_ROOT
for q in "c3_slab 6" "c3_slab 7" "c3_stride 1" "c3_stride 2"; do
  bash $R/tools/profile_query.sh $q r06f || exit 1
done
