# round 5: whole chunks and cut chunks in separate dense launches -- parity,
# then the slab (0,) / (2,) mean queries with and without the split
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/split
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_axes_cuts.py tests/test_gpu_active.py tests/test_gpu_records.py tests/test_gpu_zero_sign.py tests/test_gpu_golden.py > $O/tests.log 2>&1 || exit 1
cd /tmp
for q in 4 5; do
  for sp in 1 0; do
    rm -rf /tmp/zp
    PYAS_CUT_SPLIT=$sp timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zp -o run -- python3 $R/tools/query_c3.py c3_slab $q --reps 20 > $O/slab_${q}_split$sp.json 2> $O/slab_${q}_split$sp.err || exit 1
    cp $(find /tmp/zp -name '*kernel_stats.csv' | head -n 1) $O/slab_${q}_split${sp}_kernel_stats.csv
  done
done
