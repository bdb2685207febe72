# round 4: aligned hyperslab rows through run_rows_any too
set -o pipefail
O=gpurun_out/r04/rows7
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests -m gpu -k "golden or select or storage or fullsize or hyperslab or active or coalesc or zero_sign" > $O/tests.log 2>&1 || exit 1
for ix in 4:1020 1:1023 0:1023 0:1024; do
  timeout -k 10 300 python -u tools/bench_zeros.py --zeros 0 --axes none --reps 9 --index $ix > $O/idx_$ix.json 2> $O/idx_$ix.err || exit 1
done
timeout -k 10 400 python -u bench.py --config c5 --extra none > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
