# round 5: LDS row layout lanes per output (PYAS_ROW_LDS) x tiles per wave
# (PYAS_ROW_LDS_TPW) on C3 (2,) compact records, plain chunks
set -o pipefail
O=gpurun_out/r05/rowlds
mkdir -p $O
for h in 1 2 4; do
  for tpw in 1 2; do
    PYAS_ROW_LDS=$h PYAS_ROW_LDS_TPW=$tpw timeout -k 10 200 python -u tools/bench_axes.py --rec sum --only 2 > $O/h${h}_t${tpw}.json 2> $O/h${h}_t${tpw}.err || exit 1
  done
done
