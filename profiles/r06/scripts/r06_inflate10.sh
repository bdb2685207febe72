# round 6: decoder walk with two chain steps per loop test (variant lib), and
# NG 8 (512-bit windows, 150 VGPRs) on the main lib
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/inflate10
mkdir -p $O
cd $R
timeout -k 10 300 python -u tools/bench_inflate.py --sweep 1,30,256 > $O/bench_ng4.json 2> $O/bench_ng4.err || exit 1
PYAS_LIB=$R/pyactivestorage_amd/lib/walk2/libpyas_walk2.so timeout -k 10 300 python -u tools/bench_inflate.py --sweep 1,30,256 > $O/bench_walkpairs_ng4.json 2> $O/bench_walkpairs_ng4.err || exit 1
PYAS_INFLATE_NG=8 timeout -k 10 300 python -u tools/bench_inflate.py --sweep 1,30,256 > $O/bench_ng8.json 2> $O/bench_ng8.err || exit 1
PYAS_INFLATE_NG=8 PYAS_LIB=$R/pyactivestorage_amd/lib/walk2/libpyas_walk2.so timeout -k 10 300 python -u tools/bench_inflate.py --sweep 1,256 > $O/bench_walkpairs_ng8.json 2> $O/bench_walkpairs_ng8.err || exit 1
# the keyed grid combine with 32-bit keys: zero-sign tests, then slab (2,)
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_zero_sign.py tests/test_gpu_axes_cuts.py tests/test_gpu_records.py tests/test_gpu_sharded.py > $O/zs_tests.log 2>&1 || exit 1
cd /tmp
for m in mean min; do
  for z in 0.02 0.5; do
    tag=c3_slab_7_${m}_z$z
    rm -rf /tmp/zp
    timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zp -o run -- python3 $R/tools/query_c3.py c3_slab 7 --method $m --zeros $z --reps 10 > $O/$tag.json 2> $O/$tag.err || exit 1
    cp $(find /tmp/zp -name '*kernel_stats.csv' | head -n 1) $O/${tag}_kernel_stats.csv
  done
done
