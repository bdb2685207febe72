# round 6: zero sign after the table pick in the LDS row walk and level 2
# keyed in the grid combine -- the zero-sign and axes tests, then slab and
# whole (2,) min against mean on the same (fill-only) variable
set -o pipefail
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
O=$R/gpurun_out/r06/zeros2
mkdir -p $O
cd $R
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_zero_sign.py tests/test_gpu_axes_cuts.py tests/test_gpu_axes_rowlds.py tests/test_gpu_axes_slab.py tests/test_gpu_records.py tests/test_gpu_active.py > $O/tests.log 2>&1 || exit 1
cd /tmp
for q in "c3_slab 7" "c3_slab 6" "c3_whole 2"; do
  set -- $q
  for z in 0.02 0.5; do
    for m in mean min; do
      tag=${1}_${2}_${m}_z$z
      rm -rf /tmp/zp
      timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zp -o run -- python3 $R/tools/query_c3.py $1 $2 --method $m --zeros $z --reps 10 > $O/$tag.json 2> $O/$tag.err || exit 1
      cp $(find /tmp/zp -name '*kernel_stats.csv' | head -n 1) $O/${tag}_kernel_stats.csv
    done
  done
done
cd $R
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_inflate.py > $O/inflate_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_inflate.py --sweep 1,30,256 > $O/inflate_bench.json 2> $O/inflate_bench.err || exit 1
PYAS_LIB=$R/pyactivestorage_amd/lib/prof/libpyas_prof.so timeout -k 10 300 python -u tools/bench_inflate.py --chunks 4 --reps 1 > $O/inflate_prof.txt 2>&1 || exit 1
