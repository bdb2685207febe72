# run_plain: wave-contiguous loads (wc variant) vs the product mapping, C3 and C2, alternating
set -o pipefail
O=gpurun_out/r03/wc
mkdir -p $O
V=$PWD/pyactivestorage_amd/lib/variants
B="python -u bench.py --extra none --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0"
timeout -k 10 300 env PYAS_LIB=$V/libpyas_wc.so python -u -m pytest -x -q --timeout 200 --timeout-method thread tests/test_gpu_golden.py tests/test_gpu_chained.py > $O/tests_wc.log 2>&1 || exit 1
for r in 1 2 3; do for c in c3 c2; do
  timeout -k 10 200 $B --config $c > $O/${c}_default_$r.json 2>&1 || exit 1
  PYAS_LIB=$V/libpyas_wc.so timeout -k 10 200 $B --config $c > $O/${c}_wc_$r.json 2>&1 || exit 1
done; done
