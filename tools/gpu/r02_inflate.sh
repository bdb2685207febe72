# inflate rewrite: parity (bit-exact vs zlib, error cases, reference HDF5 chunks), throughput sweep, phase timing
set -o pipefail
mkdir -p gpurun_out/r02i
timeout -k 10 300 python -u -m pytest -x -q --timeout 60 --timeout-method thread tests/test_gpu_inflate.py tests/test_gpu_active_files.py > gpurun_out/r02i/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_inflate.py --chunks 2048 --sweep 32,1024 --cpu-threads 1 > gpurun_out/r02i/bench.json 2> gpurun_out/r02i/bench.err || exit 2
PYAS_LIB=pyactivestorage_amd/lib/libpyas_hip_prof0.so timeout -k 10 120 python -u tools/bench_inflate.py --chunks 32 --reps 1 > gpurun_out/r02i/prof.txt 2>&1 || exit 3
