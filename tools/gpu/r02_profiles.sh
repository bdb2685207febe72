# r02 rocprofv3 evidence: bench configs (kernel stats + FETCH_SIZE + WRITE_SIZE passes)
# and the partial-axis kernels (plain / shuffled / folded)
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/profiles/r02
for cfg in c3 c2 c4 c5; do
  bash tools/profile_config.sh $cfg r02 --extra none > gpurun_out/profiles/r02/${cfg}_profile.log 2>&1 || exit 1
done
root=$PWD
cd /tmp
for mode in shuffle fold foldshuffle plain; do
  case $mode in
    shuffle) args="--shuffle";; fold) args="--fold";; foldshuffle) args="--fold --shuffle";; plain) args="";;
  esac
  out=/tmp/axprof_$mode
  rm -rf $out
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $out/trace -o run -- python3 $root/tools/bench_axes.py $args > $root/gpurun_out/profiles/r02/axes_${mode}_trace.log 2>&1 || exit 2
  timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d $out/fetch -o run -- python3 $root/tools/bench_axes.py $args > $root/gpurun_out/profiles/r02/axes_${mode}_fetch.log 2>&1 || exit 3
  cp $(find $out/trace -name '*kernel_stats.csv' | head -n 1) $root/gpurun_out/profiles/r02/axes_${mode}_kernel_stats.csv
  cp $(find $out/fetch -name '*counter_collection.csv' | head -n 1) $root/gpurun_out/profiles/r02/axes_${mode}_pmc_fetch_size.csv
done
