# k_reduce tile size sweep on C3 (bench.py --tile-bytes), two repeats
set -o pipefail
O=gpurun_out/r03/tiles
mkdir -p $O
for rep in 1 2; do for t in 0 131072 524288 1048576; do
  timeout -k 10 200 python -u bench.py --extra none --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 --tile-bytes $t > $O/t_${t}_$rep.json 2>&1 || exit 1
done; done
