# round 6: rocprofv3 stats + FETCH/WRITE for the bench's query shapes on the final tree
set -o pipefail
R=$GRAFT_REPO_ROOT
for q in "c3_slab 0" "c3_slab 3" "c3_slab 4" "c3_slab 5" "c3_slab 6" "c3_slab 7" "c3_stride 0" "c3_stride 1" "c3_stride 2" "c3_stride 3" "c3_stride 4"; do
  bash $R/tools/profile_query.sh $q r06 || exit 1
done
