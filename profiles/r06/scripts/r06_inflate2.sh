# round 6: two-wave inflate (decoder wave + writer wave per stream) --
# bit-exact tests, rates for NG = 1/2/4, phase profile of the -DPYAS_INFLATE_PROF build
set -o pipefail
O=gpurun_out/r06/inflate2
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_inflate.py > $O/tests.log 2>&1 || exit 1
for ng in 2 1 4; do
  PYAS_INFLATE_NG=$ng timeout -k 10 300 python -u tools/bench_inflate.py --sweep 1,30,256 > $O/bench_ng$ng.json 2> $O/bench_ng$ng.err || exit 1
done
for ng in 2 4; do
PYAS_INFLATE_NG=$ng PYAS_LIB=$GRAFT_REPO_ROOT/pyactivestorage_amd/lib/prof/libpyas_prof.so timeout -k 10 300 python -u tools/bench_inflate.py --chunks 4 --reps 1 > $O/prof_ng$ng.txt 2>&1 || exit 1
done
