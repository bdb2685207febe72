# round 6: the LDS row walk picks a sparse zero row's winner from a
# per-position rank table; zero-sign and axes tests, then slab (2,) pairs
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/zeros3
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_zero_sign.py tests/test_gpu_axes_cuts.py tests/test_gpu_axes_rowlds.py tests/test_gpu_axes_slab.py tests/test_gpu_records.py tests/test_gpu_active.py tests/test_gpu_inflate.py > $O/tests.log 2>&1 || exit 1
cd /tmp
for q in "c3_slab 5 mean" "c3_slab 7 min"; do
  set -- $q
  for z in 0.02 0.5; do
    tag=${1}_${2}_${3}_z$z
    rm -rf /tmp/zp
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zp -o run -- python3 $R/tools/query_c3.py $1 $2 --method $3 --zeros $z --reps 10 > $O/$tag.json 2> $O/$tag.err || exit 1
    cp $(find /tmp/zp -name '*kernel_stats.csv' | head -n 1) $O/${tag}_kernel_stats.csv
  done
done
