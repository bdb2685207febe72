# round 4: two-step zero-sign scan (hyperslab queries): a lane per output for short calls vs 16 lanes (PYAS_TIE_GROUP=16)
set -o pipefail
O=gpurun_out/r04/zeros9
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_zero_sign.py tests/test_gpu_golden.py > $O/tests.log 2>&1 || exit 1
for g in "" 16; do
  PYAS_TIE_GROUP=$g timeout -k 10 300 python -u tools/bench_zeros.py --zeros 0.5 --axes none,0,2 --reps 5 --index 1:1023 > $O/idx_g$g.json 2> $O/idx_g$g.err || exit 1
done
(cd /tmp && rm -rf /tmp/zt && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zt -o run -- \
   python3 $R/tools/bench_zeros.py --zeros 0.5 --axes none,0,2 --reps 5 --index 1:1023 > $R/$O/idx_prof.log 2>&1) || exit 1
cp $(find /tmp/zt -name '*kernel_stats.csv' | head -n 1) $O/idx_kernel_stats.csv
timeout -k 10 300 python -u tools/bench_zeros.py --zeros 0 --axes none,0,2 --reps 5 --index 1:1023 > $O/idx_zeros0.json 2> $O/idx_zeros0.err || exit 1
