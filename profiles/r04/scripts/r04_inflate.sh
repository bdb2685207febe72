# round 4: inflate output step without LDS marks/scan -- parity, then the
# per-stream and 2048-stream rates against the round-3 kernel (lib/before)
set -o pipefail
O=gpurun_out/r04/inflate
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_inflate.py > $O/tests.log 2>&1 || exit 1
for lib in new before; do
  if [ $lib = before ]; then export PYAS_LIB=$R/pyactivestorage_amd/lib/before/libpyas_before.so; else unset PYAS_LIB; fi
  timeout -k 10 300 python -u tools/bench_inflate.py --sweep 1,8,30,256 > $O/bench_$lib.json 2> $O/bench_$lib.err || exit 1
done
