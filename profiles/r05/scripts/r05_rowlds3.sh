# round 5: two tiles per wave for whole-chunk / zero-sign LDS rows -- parity,
# then C3 (2,) records under rocprofv3 and the slab (2,) queries
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/rowlds3
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_axes_rowlds.py tests/test_gpu_axes_dense.py tests/test_gpu_zero_sign.py tests/test_gpu_records.py tests/test_gpu_axes_cuts.py > $O/tests.log 2>&1 || exit 1
cd /tmp
rm -rf /tmp/ap
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ap -o run -- python3 $R/tools/bench_axes.py --rec sum --only 2 > $O/plainrec_2.json 2> $O/plainrec_2.err || exit 1
cp $(find /tmp/ap -name '*kernel_stats.csv' | head -n 1) $O/plainrec_2_kernel_stats.csv
for m in mean min; do
  timeout -k 10 200 python3 $R/tools/query_c3.py c3_slab 5 --method $m --reps 20 > $O/slab_${m}.json 2> $O/slab_${m}.err || exit 1
done
