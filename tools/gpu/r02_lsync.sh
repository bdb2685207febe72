# lean fold: block barrier every 1 / 4 load groups (waves of a block kept in step) vs none, C3 fold
set -o pipefail
mkdir -p gpurun_out/r02f
for rep in 1 2; do
for v in default lsync1 lsync4; do
  if [ $v = default ]; then lib=""; else lib=$PWD/pyactivestorage_amd/lib/variants/libpyas_$v.so; fi
  for mode in "--fold" "--fold --shuffle"; do
    PYAS_LIB=$lib timeout -k 10 120 python -u tools/bench_axes.py $mode | sed "s/^/$v /" >> gpurun_out/r02f/lsync.txt 2>> gpurun_out/r02f/lsync.err || exit 1
  done
done
done
