# round 5: grid combine with 8-B record loads, 16 layers in flight -- parity, kernel splits
# of the slab (0,) / (2,) mean queries
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/comb
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_records.py tests/test_gpu_zero_sign.py tests/test_gpu_axes_fold.py tests/test_gpu_active.py tests/test_gpu_golden.py > $O/tests.log 2>&1 || exit 1
cd /tmp
for q in 4 5; do
  rm -rf /tmp/zp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zp -o run -- python3 $R/tools/query_c3.py c3_slab $q --reps 10 > $O/slab_$q.json 2> $O/slab_$q.err || exit 1
  cp $(find /tmp/zp -name '*kernel_stats.csv' | head -n 1) $O/slab_${q}_kernel_stats.csv
done
