# chunks per workgroup around the auto choice: plain (0,) (NV 4) and (1,) (NV 2), C3, two repeats
set -o pipefail
O=gpurun_out/r03/cpb
mkdir -p $O
for r in 1 2; do
  for c in 1 2 3 4 6; do PYAS_COL_STREAM=$c timeout -k 10 120 python -u tools/bench_axes.py --only 0 > $O/a0_${c}_$r.json 2>&1 || exit 1; done
  for c in 16 24 32 48 64; do PYAS_COL_STREAM=$c timeout -k 10 120 python -u tools/bench_axes.py --only 1 > $O/a1_${c}_$r.json 2>&1 || exit 1; done
done
