# round 5: LDS row tiles per wave (PYAS_ROW_LDS_TPW) confirmation -- C3 (2,)
# per-chunk records (twice each), then the slab (2,) mean / min queries
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/rowlds2
mkdir -p $O
for rep in a b; do
  for tpw in 1 2 3 4; do
    PYAS_ROW_LDS_TPW=$tpw timeout -k 10 200 python -u tools/bench_axes.py --rec sum --only 2 > $O/t${tpw}_$rep.json 2> $O/t${tpw}_$rep.err || exit 1
  done
done
for tpw in 1 2; do
  for m in mean min; do
    PYAS_ROW_LDS_TPW=$tpw timeout -k 10 200 python3 $R/tools/query_c3.py c3_slab 5 --method $m --reps 20 > $O/slab_${m}_t$tpw.json 2> $O/slab_${m}_t$tpw.err || exit 1
  done
done
