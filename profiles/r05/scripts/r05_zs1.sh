# round 5: zero-sign cost on the two-step path ([1:1023]^3, 50 % and 2 % zeros) and spans A/B
set -o pipefail
O=gpurun_out/r05/zs1
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread $R/tests/test_gpu_spans.py > $R/$O/spans_tests.log 2>&1 || exit 1
for z in 0.5 0.02 0; do
  for q in 0 4 5; do
    rm -rf /tmp/zp
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zp -o run -- python3 $R/tools/query_c3.py c3_slab $q --method min --zeros $z --reps 10 > $R/$O/min_${q}_z$z.json 2> $R/$O/min_${q}_z$z.err || exit 1
    cp $(find /tmp/zp -name '*kernel_stats.csv' | head -n 1) $R/$O/min_${q}_z${z}_kernel_stats.csv
  done
done
cd $R
for sp in 1 2; do
  PYAS_SPANS=$sp timeout -k 10 400 python -u bench.py --steps 10 --extra c5,c3_slab --extra-steps 10 --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 > $O/bench_spans$sp.json 2> $O/bench_spans$sp.err || exit 1
done
