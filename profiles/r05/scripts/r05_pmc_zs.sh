# round 5: instruction mix of the LDS row zero-sign kernel against the cut kernel
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r05/pmc_zs
mkdir -p $O
cd /tmp
for m in min mean; do
  rm -rf /tmp/pz
  timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_WAVE_CYCLES SQ_INSTS_VMEM_RD SQ_WAVES SQ_BUSY_CYCLES SQ_INSTS_SMEM --output-format csv -d /tmp/pz -o run -- python3 $R/tools/query_c3.py c3_slab 5 --method $m --reps 3 > $O/$m.json 2> $O/$m.err || exit 1
  cp $(find /tmp/pz -name '*counter_collection.csv' | head -n 1) $O/${m}_counters.csv
done
