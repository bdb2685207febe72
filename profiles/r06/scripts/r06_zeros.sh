# round 6: zero-sign cost against the SAME variable's mean
# (fill-only attrs, as every --zeros field): slab and whole (2,) and (0,),
# full reductions; e2e medians and rocprof kernel splits
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/zeros
mkdir -p $O
cd /tmp
for q in "c3_slab 7" "c3_slab 6" "c3_whole 2" "c3_whole 1" "c3_whole 0"; do
  set -- $q
  for z in 0.02 0.5; do
    for m in mean min; do
      tag=${1}_${2}_${m}_z$z
      rm -rf /tmp/zp
      timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zp -o run -- python3 $R/tools/query_c3.py $1 $2 --method $m --zeros $z --reps 10 > $O/$tag.json 2> $O/$tag.err || exit 1
      cp $(find /tmp/zp -name '*kernel_stats.csv' | head -n 1) $O/${tag}_kernel_stats.csv
    done
  done
done
