# round 5: tile bytes (workgroups per chunk) for sparse selections: the
# 64-entry list and the stride-3 rows, end to end
set -o pipefail
O=gpurun_out/r05/tiles
mkdir -p $O
for tb in 0 131072 65536 32768; do
  for q in 2 0; do
    timeout -k 10 200 python3 tools/query_c3.py c3_stride $q --reps 20 --tile-bytes $tb > $O/stride_${q}_tb$tb.json 2> $O/stride_${q}_tb$tb.err || exit 1
  done
  timeout -k 10 200 python3 tools/query_c3.py c3_slab 0 --reps 20 --tile-bytes $tb > $O/slab_0_tb$tb.json 2> $O/slab_0_tb$tb.err || exit 1
done
