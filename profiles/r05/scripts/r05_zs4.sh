# round 5: 32-bit grid-combine decode, zero-row pass re-reading the tile;
# parity, then slab (0,)/(2,) kernel splits and the row kernels' instruction mix
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/zs4
mkdir -p $O
T="python -u -m pytest -x -q --timeout 200 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_zero_sign.py tests/test_gpu_axes_cuts.py tests/test_gpu_active.py tests/test_gpu_axes_fold.py tests/test_gpu_records.py > $O/tests.log 2>&1 || exit 1
cd /tmp
prof() {   # name which method zeros tag
  rm -rf /tmp/zp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zp -o run -- python3 $R/tools/query_c3.py $1 $2 --method $3 --zeros $4 --reps 10 > $O/$5.json 2> $O/$5.err || return 1
  cp $(find /tmp/zp -name '*kernel_stats.csv' | head -n 1) $O/$5_kernel_stats.csv
}
prof c3_slab 4 mean 0 slab_mean_0 || exit 1
prof c3_slab 5 mean 0 slab_mean_2 || exit 1
for z in 0 0.02 0.5; do
  prof c3_slab 5 min $z slab_min_2_z$z || exit 1
done
for m in min mean; do
  rm -rf /tmp/pz
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SMEM --output-format csv -d /tmp/pz -o run -- python3 $R/tools/query_c3.py c3_slab 5 --method $m --reps 3 > $O/pmc_$m.json 2> $O/pmc_$m.err || exit 1
  cp $(find /tmp/pz -name '*counter_collection.csv' | head -n 1) $O/pmc_${m}_counters.csv
done
