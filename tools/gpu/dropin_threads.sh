set -o pipefail
mkdir -p gpurun_out/r02
for t in 4 8 16 30 64; do
  timeout -k 10 120 python -u tools/bench_dropin.py --chunks 8192 --threads $t --gpu-only --trials 5 --ceiling-read >> gpurun_out/r02/dropin_threads.jsonl 2>> gpurun_out/r02/dropin_threads.err || exit 1
done
