# round 5: walk-keyed level-1 zero sign -- parity, then the zero-heavy two-step costs
set -o pipefail
O=gpurun_out/r05/zs2
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_zero_sign.py tests/test_gpu_records.py tests/test_gpu_axes_cuts.py tests/test_gpu_spans.py tests/test_gpu_active.py > $O/tests.log 2>&1 || exit 1
cd /tmp
for z in 0.5 0.02 0; do
  for q in 1 4 5; do
    rm -rf /tmp/zp
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zp -o run -- python3 $R/tools/query_c3.py c3_slab $q --method min --zeros $z --reps 10 > $R/$O/min_${q}_z$z.json 2> $R/$O/min_${q}_z$z.err || exit 1
    cp $(find /tmp/zp -name '*kernel_stats.csv' | head -n 1) $R/$O/min_${q}_z${z}_kernel_stats.csv
  done
done
