set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 300 python -u -m pytest -x -q --timeout 300 --timeout-method thread -s tests/test_gpu_coalesced.py tests/test_fastpath.py > gpurun_out/r02/test_coalesced.log 2>&1 || exit 2
for t in 8 30; do
  timeout -k 10 120 python -u tools/bench_dropin.py --chunks 8192 --threads $t --gpu-only --trials 5 --ceiling-us 400 >> gpurun_out/r02/dropin_sweep.jsonl 2>> gpurun_out/r02/dropin_sweep.err || exit 1
done
timeout -k 10 300 python -u tools/bench_dropin.py --chunks 8192 > gpurun_out/r02/dropin_bench.json 2> gpurun_out/r02/dropin_bench.err || exit 3
