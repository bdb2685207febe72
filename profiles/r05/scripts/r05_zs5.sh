# round 5: the row fold gathers zero bits in its main pass -- parity, then the
# whole-variable (2,) min at 0 / 2 / 50 % zeros and mean
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/zs5
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_zero_sign.py tests/test_gpu_axes_fold.py tests/test_gpu_axes_rowlds.py tests/test_gpu_golden.py > $O/tests.log 2>&1 || exit 1
cd /tmp
for z in 0 0.02 0.5; do
  rm -rf /tmp/zp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zp -o run -- python3 $R/tools/query_c3.py c3_whole 2 --method min --zeros $z --reps 10 > $O/whole_min_2_z$z.json 2> $O/whole_min_2_z$z.err || exit 1
  cp $(find /tmp/zp -name '*kernel_stats.csv' | head -n 1) $O/whole_min_2_z${z}_kernel_stats.csv
done
rm -rf /tmp/zp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zp -o run -- python3 $R/tools/query_c3.py c3_whole 2 --method mean --reps 10 > $O/whole_mean_2.json 2> $O/whole_mean_2.err || exit 1
cp $(find /tmp/zp -name '*kernel_stats.csv' | head -n 1) $O/whole_mean_2_kernel_stats.csv
