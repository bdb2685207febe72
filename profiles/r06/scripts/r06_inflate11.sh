# round 6: decoder windows past the first 32 KiB take one wave sum (no per-token offsets)
# dword writes
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/inflate11
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_inflate.py tests/test_gpu_active_files.py tests/test_gpu_ingest.py > $O/inflate_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_inflate.py --sweep 1,30,256 > $O/bench.json 2> $O/bench.err || exit 1
PYAS_LIB=$R/pyactivestorage_amd/lib/prof/libpyas_prof.so timeout -k 10 300 python -u tools/bench_inflate.py --chunks 4 --reps 1 > $O/prof.txt 2>&1 || exit 1
