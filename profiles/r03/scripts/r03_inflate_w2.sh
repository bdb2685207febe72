# inflate: two output positions per lane per step (W2) vs one (iw1 variant): parity, throughput, Active zlib E2E
set -o pipefail
O=gpurun_out/r03/w2
mkdir -p $O
V=$PWD/pyactivestorage_amd/lib/variants
timeout -k 10 400 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_inflate.py > $O/tests.log 2>&1 || exit 1
for rep in 1 2; do
  timeout -k 10 200 python -u tools/bench_inflate.py --chunks 2048 --sweep 32,256 > $O/w2_$rep.json 2> $O/w2_$rep.err || exit 1
  PYAS_LIB=$V/libpyas_iw1.so timeout -k 10 200 python -u tools/bench_inflate.py --chunks 2048 --sweep 32,256 > $O/w1_$rep.json 2> $O/w1_$rep.err || exit 1
done
timeout -k 10 300 python -u tools/bench_active.py --zlib > $O/active_zlib_w2.json 2> $O/active_zlib_w2.err || exit 1
PYAS_LIB=$V/libpyas_iw1.so timeout -k 10 300 python -u tools/bench_active.py --zlib > $O/active_zlib_w1.json 2> $O/active_zlib_w1.err || exit 1
