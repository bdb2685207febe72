# inflate rewrite end to end: parity (inflate, files, golden, coalesced), kernel rate, Active zlib query by group count, zlib drop-in
set -o pipefail
mkdir -p gpurun_out/r02e
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_inflate.py tests/test_gpu_active_files.py tests/test_gpu_golden.py tests/test_gpu_coalesced.py tests/test_gpu_active.py > gpurun_out/r02e/tests.log 2>&1 || exit 1
timeout -k 10 200 python -u tools/bench_inflate.py --chunks 2048 --sweep 32,1024,4096 --cpu-threads 16 > gpurun_out/r02e/inflate_bench.json 2> gpurun_out/r02e/inflate_bench.err || exit 2
for g in 4 2 8; do
  PYAS_INFLATE_GROUPS=$g timeout -k 10 300 python -u tools/bench_active.py --zlib --axes none --reps 3 > gpurun_out/r02e/active_zlib_g$g.json 2> gpurun_out/r02e/active_zlib_g$g.err || exit 3
done
timeout -k 10 300 python -u tools/bench_dropin.py --zlib --chunks 1024 --percall-chunks 256 --trials 3 > gpurun_out/r02e/dropin_zlib.json 2> gpurun_out/r02e/dropin_zlib.err || exit 4
