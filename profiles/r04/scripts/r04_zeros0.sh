# round 4, first measurement: zero-sign pass cost on zero-heavy data (before),
# plus the per-chunk axes sweep on the round-3 final library (grid rule d7df369)
set -o pipefail
O=gpurun_out/r04/zeros0
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_zero_sign.py -x -q --timeout 250 --timeout-method thread > $O/zs_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_zeros.py --zeros 0.5 --axes none,0,2 --reps 5 > $O/zeros50.json 2> $O/zeros50.err || exit 1
timeout -k 10 300 python -u tools/bench_zeros.py --zeros 0 --axes none,0,2 --reps 5 > $O/zeros0.json 2> $O/zeros0.err || exit 1
cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zt -o run -- \
   python3 $GRAFT_REPO_ROOT/tools/bench_zeros.py --zeros 0.5 --axes none,0,2 --reps 5 > $GRAFT_REPO_ROOT/$O/zeros50_prof.log 2>&1 || exit 1
cd $GRAFT_REPO_ROOT
cp $(find /tmp/zt -name '*kernel_stats.csv' | head -n 1) $O/zeros50_kernel_stats.csv
timeout -k 10 300 python -u tools/bench_axes.py > $O/axes_plain.json 2> $O/axes_plain.err || exit 1
timeout -k 10 300 python -u tools/bench_axes.py --shuffle > $O/axes_shuf.json 2> $O/axes_shuf.err || exit 1
