# round 6: Active inflate crossover, host lanes spread over the staging slots,
# one device launch per <= 2048 streams
set -o pipefail
O=gpurun_out/r06/xover
mkdir -p $O
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_inflate.py tests/test_gpu_active_files.py tests/test_gpu_ingest.py tests/test_gpu_resident.py > $O/tests_files.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_inflate_crossover.py --ks 1,4,16,32,64,128,192,256,384,512,768,1024 > $O/crossover.json 2> $O/crossover.err || exit 1
