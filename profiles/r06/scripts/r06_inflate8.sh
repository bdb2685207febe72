# round 6: token queue without output offsets (1024 tokens in the same LDS),
# stored blocks with four 1 KiB steps of input loads in flight; a 2048-token
# variant; then the zero-sign slab (2,) after reverting the table pick and
# keying the grid combine only when asked
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/inflate8
mkdir -p $O
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_inflate.py tests/test_gpu_active_files.py > $O/inflate_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_inflate.py --sweep 1,30,256 > $O/bench_q1024.json 2> $O/bench_q1024.err || exit 1
PYAS_LIB=$R/pyactivestorage_amd/lib/q2048/libpyas_q2048.so timeout -k 10 300 python -u tools/bench_inflate.py --sweep 1,30,256 > $O/bench_q2048.json 2> $O/bench_q2048.err || exit 1
PYAS_LIB=$R/pyactivestorage_amd/lib/prof/libpyas_prof.so timeout -k 10 300 python -u tools/bench_inflate.py --chunks 4 --reps 1 > $O/prof_q1024.txt 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_zero_sign.py tests/test_gpu_axes_cuts.py tests/test_gpu_axes_rowlds.py > $O/zs_tests.log 2>&1 || exit 1
cd /tmp
for m in mean min; do
  for z in 0.02 0.5; do
    tag=c3_slab_7_${m}_z$z
    rm -rf /tmp/zp
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zp -o run -- python3 $R/tools/query_c3.py c3_slab 7 --method $m --zeros $z --reps 10 > $O/$tag.json 2> $O/$tag.err || exit 1
    cp $(find /tmp/zp -name '*kernel_stats.csv' | head -n 1) $O/${tag}_kernel_stats.csv
  done
done
