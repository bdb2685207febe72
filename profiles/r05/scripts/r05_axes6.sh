# round 5: per-chunk partial-axis kernels and the LDS row
# zero-sign kernel: kernel stats for plain (2,) / shuffled (1,) records, the
# slab (2,) min at 0 / 2 / 50 % zeros, parity of the touched tests first
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/axes6
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_zero_sign.py tests/test_gpu_axes_cuts.py tests/test_gpu_axes_slab.py tests/test_gpu_records.py > $O/tests.log 2>&1 || exit 1
cd /tmp
for spec in "plainrec:2" "shufrec:1" "plainrec:0"; do
  kind=${spec%%:*}; ax=${spec#*:}
  case $kind in plainrec) a="--rec sum";; shufrec) a="--shuffle --rec sum";; esac
  tag=${kind}_$ax
  rm -rf /tmp/ap
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/ap/trace -o run -- python3 $R/tools/bench_axes.py $a --only $ax > $O/${tag}_trace.log 2>&1 || exit 1
  cp $(find /tmp/ap/trace -name '*kernel_stats.csv' | head -n 1) $O/${tag}_kernel_stats.csv
done
for z in 0 0.02 0.5; do
  rm -rf /tmp/zp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zp -o run -- python3 $R/tools/query_c3.py c3_slab 5 --method min --zeros $z --reps 10 > $O/slab_min_2_z$z.json 2> $O/slab_min_2_z$z.err || exit 1
  cp $(find /tmp/zp -name '*kernel_stats.csv' | head -n 1) $O/slab_min_2_z${z}_kernel_stats.csv
done
rm -rf /tmp/zp
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zp -o run -- python3 $R/tools/query_c3.py c3_slab 5 --reps 10 > $O/slab_mean_2.json 2> $O/slab_mean_2.err || exit 1
cp $(find /tmp/zp -name '*kernel_stats.csv' | head -n 1) $O/slab_mean_2_kernel_stats.csv
