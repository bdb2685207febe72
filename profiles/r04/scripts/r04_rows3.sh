# round 4: hyperslab full reductions -- which path costs what (aligned rows vs any-alignment runs), PMC of k_reduce_u
set -o pipefail
O=gpurun_out/r04/rows3
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
for ix in 4:1020 1:1023 0:1023 0:1024; do
  timeout -k 10 300 python -u tools/bench_zeros.py --zeros 0 --axes none --reps 9 --index $ix > $O/idx_$ix.json 2> $O/idx_$ix.err || exit 1
done
cd /tmp
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/r3/fetch -o run -- python3 $R/tools/bench_zeros.py --zeros 0 --axes none --reps 3 --index 1:1023 > $R/$O/fetch.log 2>&1 || exit 1
timeout -s KILL 200 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_VMEM_RD SQ_WAVES SQ_WAVE_CYCLES --output-format csv -d /tmp/r3/sq -o run -- python3 $R/tools/bench_zeros.py --zeros 0 --axes none --reps 3 --index 1:1023 > $R/$O/sq.log 2>&1 || exit 1
cp $(find /tmp/r3/fetch -name '*counter_collection.csv' | head -n 1) $R/$O/fetch.csv
cp $(find /tmp/r3/sq -name '*counter_collection.csv' | head -n 1) $R/$O/sq.csv
