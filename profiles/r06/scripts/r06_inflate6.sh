# round 6: table-folded stop conditions; decoder-alone diagnostic (writer skips tokens)
set -o pipefail
O=gpurun_out/r06/inflate6
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_inflate.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_inflate.py --sweep 1,30,256 > $O/bench_ng4.json 2> $O/bench_ng4.err || exit 1
PYAS_LIB=$GRAFT_REPO_ROOT/pyactivestorage_amd/lib/prof/libpyas_prof.so timeout -k 10 300 python -u tools/bench_inflate.py --chunks 4 --reps 1 > $O/prof_ng4.txt 2>&1 || exit 1
PYAS_LIB=$GRAFT_REPO_ROOT/pyactivestorage_amd/lib/prof2/libpyas_prof2.so timeout -k 10 300 python -u tools/bench_inflate.py --chunks 4 --reps 1 --no-check > $O/prof_deconly_ng4.txt 2>&1 || exit 1
PYAS_LIB=$GRAFT_REPO_ROOT/pyactivestorage_amd/lib/prof2/libpyas_prof2.so timeout -k 10 300 python -u tools/bench_inflate.py --no-check --sweep 1 > $O/bench_deconly_ng4.json 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_active_files.py tests/test_gpu_ingest.py > $O/tests_files.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_inflate_crossover.py > $O/crossover.json 2> $O/crossover.err || exit 1
