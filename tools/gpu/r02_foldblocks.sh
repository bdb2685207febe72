set -o pipefail
mkdir -p gpurun_out/r02
for b in 2048 1024 512; do
  for mode in "--fold" "--fold --shuffle"; do
    timeout -k 10 120 python -u tools/bench_axes.py $mode --fold-blocks $b | sed "s/^/$b /" >> gpurun_out/r02/foldblocks.txt 2>> gpurun_out/r02/foldblocks.err || exit 1
  done
done
