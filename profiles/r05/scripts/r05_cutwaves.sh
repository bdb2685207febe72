# round 5: the cut row kernel at 3 waves (no scratch) against 4 (12 B scratch),
# slab (2,) mean, same box, alternating
set -o pipefail
O=gpurun_out/r05/cutwaves
mkdir -p $O
for rep in a b; do
  timeout -k 10 200 python3 tools/query_c3.py c3_slab 5 --reps 30 > $O/w4_$rep.json 2> $O/w4_$rep.err || exit 1
  PYAS_LIB=$PWD/pyactivestorage_amd/lib/exp/libpyas_cut3.so timeout -k 10 200 python3 tools/query_c3.py c3_slab 5 --reps 30 > $O/w3_$rep.json 2> $O/w3_$rep.err || exit 1
done
