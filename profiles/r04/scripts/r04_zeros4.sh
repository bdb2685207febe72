# round 4: zero bits built in the row fold's main pass, scalar level-2 keys
set -o pipefail
O=gpurun_out/r04/zeros4
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_zero_sign.py tests/test_gpu_axes_slab.py tests/test_gpu_records.py tests/test_gpu_axes_fold.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_zeros.py --zeros 0.5 --axes none,0,2 --reps 5 > $O/zeros50.json 2> $O/zeros50.err || exit 1
timeout -k 10 300 python -u tools/bench_zeros.py --zeros 0 --axes none,0,2 --reps 5 > $O/zeros0.json 2> $O/zeros0.err || exit 1
timeout -k 10 300 python -u tools/bench_zeros.py --zeros 0.02 --axes none,0,2 --reps 5 > $O/zeros2.json 2> $O/zeros2.err || exit 1
(cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zt -o run -- \
   python3 $R/tools/bench_zeros.py --zeros 0.5 --axes none,0,2 --reps 5 > $R/$O/zeros50_prof.log 2>&1) || exit 1
cp $(find /tmp/zt -name '*kernel_stats.csv' | head -n 1) $O/zeros50_kernel_stats.csv
