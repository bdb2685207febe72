# LDS row layout tiles per wave (PYAS_ROW_LDS_TPW) with the staged partial stores, C3 per-chunk (2,)
set -o pipefail
O=gpurun_out/r03/tpw
mkdir -p $O
for rep in 1 2; do for t in 1 2 4 8 16; do
  PYAS_ROW_LDS_TPW=$t timeout -k 10 120 python -u tools/bench_axes.py --only 2 > $O/plain_${t}_$rep.json 2>&1 || exit 1
  PYAS_ROW_LDS_TPW=$t timeout -k 10 120 python -u tools/bench_axes.py --only 2 --shuffle > $O/shuf_${t}_$rep.json 2>&1 || exit 1
done; done
