# round 6: token decoder (PYAS_INFLATE_NG=1/2/4) against the round-3 windowed
# decoder (NG=0) -- bit-exact tests first, then rates on 2048 x 1 MiB streams
# and the per-stream sweep; the sharded entry's zero sign and attach tests
set -o pipefail
O=gpurun_out/r06/inflate1
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_inflate.py > $O/tests_ng4.log 2>&1 || exit 1
for ng in 0 4 2 1; do
  PYAS_INFLATE_NG=$ng timeout -k 10 300 python -u tools/bench_inflate.py --sweep 1,30,256 > $O/bench_ng$ng.json 2> $O/bench_ng$ng.err || exit 1
done
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_sharded.py tests/test_gpu_resident.py > $O/tests_shard.log 2>&1 || exit 1
