# round 6: two-symbol walk steps (decoder alone and full), then the Active
# inflate crossover with host lanes spread over the staging slots
set -o pipefail
O=gpurun_out/r06/inflate7
mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_inflate.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_inflate.py --sweep 1,30,256 > $O/bench_ng4.json 2> $O/bench_ng4.err || exit 1
PYAS_LIB=$GRAFT_REPO_ROOT/pyactivestorage_amd/lib/prof/libpyas_prof.so timeout -k 10 300 python -u tools/bench_inflate.py --chunks 4 --reps 1 > $O/prof_ng4.txt 2>&1 || exit 1
PYAS_LIB=$GRAFT_REPO_ROOT/pyactivestorage_amd/lib/prof2/libpyas_prof2.so timeout -k 10 300 python -u tools/bench_inflate.py --chunks 4 --reps 1 --no-check > $O/prof_deconly_ng4.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_active_files.py tests/test_gpu_ingest.py tests/test_gpu_resident.py > $O/tests_files.log 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_inflate_crossover.py --ks 1,4,16,32,64,128,192,256,384,512,768,1024 > $O/crossover.json 2> $O/crossover.err || exit 1
