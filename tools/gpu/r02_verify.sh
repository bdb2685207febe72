# full GPU suite, smoke, default bench and the drop-in at the default coalescer depth (one box call)
set -o pipefail
mkdir -p gpurun_out/r02v
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02v/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02v/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > gpurun_out/r02v/bench_default.json 2> gpurun_out/r02v/bench_default.err || exit 3
timeout -k 10 300 python -u tools/bench_dropin.py --chunks 4096 --trials 3 --ceiling-read > gpurun_out/r02v/dropin_bench.json 2> gpurun_out/r02v/dropin_bench.err || exit 4
timeout -k 10 300 python -u tools/bench_dropin.py --zlib --chunks 1024 --percall-chunks 256 --trials 3 > gpurun_out/r02v/dropin_bench_zlib.json 2>> gpurun_out/r02v/dropin_bench.err || exit 5
