# round 4: row-fold sign with rank tables (no VGPR floor); kernel stats at 0 %, 2 %, 50 % zeros
set -o pipefail
O=gpurun_out/r04/zeros8
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_zero_sign.py > $O/tests.log 2>&1 || exit 1
for z in 0.5 0.02 0; do
  timeout -k 10 300 python -u tools/bench_zeros.py --zeros $z --axes none,0,2 --reps 5 > $O/zeros_$z.json 2> $O/zeros_$z.err || exit 1
  (cd /tmp && rm -rf /tmp/zt && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zt -o run -- \
     python3 $R/tools/bench_zeros.py --zeros $z --axes none,0,2 --reps 5 > $R/$O/zeros_${z}_prof.log 2>&1) || exit 1
  cp $(find /tmp/zt -name '*kernel_stats.csv' | head -n 1) $O/zeros_${z}_kernel_stats.csv
done
