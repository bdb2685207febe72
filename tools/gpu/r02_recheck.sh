# box-variance recheck: per-chunk and fold axes, drop-in
set -o pipefail
mkdir -p gpurun_out/r02y
for mode in "" "--shuffle" "--fold" "--fold --shuffle"; do
  timeout -k 10 120 python -u tools/bench_axes.py $mode >> gpurun_out/r02y/axes.jsonl 2>> gpurun_out/r02y/axes.err || exit 1
done
timeout -k 10 300 python -u tools/bench_dropin.py --chunks 4096 --trials 3 --ceiling-read > gpurun_out/r02y/dropin_bench.json 2> gpurun_out/r02y/dropin_bench.err || exit 2
timeout -k 10 300 python -u bench.py --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 --extra none > gpurun_out/r02y/bench_quick.json 2> gpurun_out/r02y/bench_quick.err || exit 3
