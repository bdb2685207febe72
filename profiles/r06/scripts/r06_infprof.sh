# round 6: phase profile of the token decoder (-DPYAS_INFLATE_PROF build)
set -o pipefail
O=gpurun_out/r06/infprof
mkdir -p $O
for ng in 4 1; do
PYAS_INFLATE_NG=$ng PYAS_LIB=$GRAFT_REPO_ROOT/pyactivestorage_amd/lib/prof/libpyas_prof.so timeout -k 10 300 python -u tools/bench_inflate.py --chunks 4 --reps 1 > $O/prof_ng$ng.txt 2>&1 || exit 1
done
