# round 5: row-call keying in the LDS row walk, compare-and-select column
# tracker, level 2 in the combine -- parity, then zero-heavy kernel splits
set -o pipefail
O=gpurun_out/r05/zs3
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_zero_sign.py tests/test_gpu_records.py tests/test_gpu_axes_cuts.py tests/test_gpu_active.py tests/test_gpu_axes_slab.py > $O/tests.log 2>&1 || exit 1
cd /tmp
prof() {   # name which method zeros tag
  rm -rf /tmp/zp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zp -o run -- python3 $R/tools/query_c3.py $1 $2 --method $3 --zeros $4 --reps 10 > $R/$O/$5.json 2> $R/$O/$5.err || return 1
  cp $(find /tmp/zp -name '*kernel_stats.csv' | head -n 1) $R/$O/$5_kernel_stats.csv
}
prof c3_slab 4 mean 0 slab_mean_0 || exit 1
prof c3_slab 5 mean 0 slab_mean_2 || exit 1
for z in 0.5 0.02 0; do
  prof c3_slab 1 min $z slab_min_full_z$z || exit 1
  prof c3_slab 4 min $z slab_min_0_z$z || exit 1
  prof c3_slab 5 min $z slab_min_2_z$z || exit 1
  prof c3_whole 0 min $z whole_min_full_z$z || exit 1
  prof c3_whole 1 min $z whole_min_0_z$z || exit 1
  prof c3_whole 2 min $z whole_min_2_z$z || exit 1
done
