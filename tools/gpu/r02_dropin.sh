# pipelined coalescer with copy stream + zero-copy meta/partials: parity, then rate by knob
set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_coalesced.py tests/test_gpu_golden.py > gpurun_out/r02/coalesced_tests.log 2>&1 || exit 1
run() { env "$@" timeout -k 10 120 python -u tools/bench_dropin.py --chunks 4096 --gpu-only --trials 3 >> gpurun_out/r02/dropin_knobs.jsonl 2>> gpurun_out/r02/dropin_knobs.err; }
run PYAS_COALESCE_DEPTH=4 || exit 2
run PYAS_COALESCE_DEPTH=1 || exit 3
run PYAS_COALESCE_DEPTH=2 || exit 4
run PYAS_COALESCE_ZEROCOPY=0 || exit 5
run PYAS_COALESCE_COPY=caller || exit 7
run PYAS_COALESCE_SYNC=spin || exit 8
timeout -k 10 300 python -u tools/bench_dropin.py --chunks 4096 --trials 3 --ceiling-read > gpurun_out/r02/dropin_bench.json 2>> gpurun_out/r02/dropin_knobs.err || exit 9
timeout -k 10 300 python -u tools/bench_dropin.py --zlib --chunks 1024 --percall-chunks 256 --trials 3 > gpurun_out/r02/dropin_bench_zlib.json 2>> gpurun_out/r02/dropin_knobs.err || exit 10
