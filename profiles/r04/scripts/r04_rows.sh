# round 4: run_rows_any (hyperslab runs at any alignment) -- full GPU suite, then the hyperslab query bench
set -o pipefail
O=gpurun_out/r04/rows
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_zeros.py --zeros 0 --axes none,0,2 --reps 5 --index 1:1023 > $O/idx_zeros0.json 2> $O/idx_zeros0.err || exit 1
timeout -k 10 300 python -u tools/bench_zeros.py --zeros 0.5 --axes none,0,2 --reps 5 --index 1:1023 > $O/idx_zeros50.json 2> $O/idx_zeros50.err || exit 1
(cd /tmp && rm -rf /tmp/zt && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zt -o run -- \
   python3 $R/tools/bench_zeros.py --zeros 0.5 --axes none,0,2 --reps 5 --index 1:1023 > $R/$O/idx_prof.log 2>&1) || exit 1
cp $(find /tmp/zt -name '*kernel_stats.csv' | head -n 1) $O/idx_zeros50_kernel_stats.csv
timeout -k 10 400 python -u bench.py --config c5 --extra none > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
