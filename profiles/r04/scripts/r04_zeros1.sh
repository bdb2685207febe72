# round 4: zero-sign pass on zero-heavy data, round-3 kernel (k_tie_chunks,
# PYAS_LIB=lib/before) against the early-stopping scan (k_tie_scan); parity
# first; then the per-chunk axes sweep on this library (grid rule d7df369),
# 32-B partials and compact records
set -o pipefail
O=gpurun_out/r04/zeros1
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_zero_sign.py tests/test_gpu_sharded.py tests/test_gpu_records.py tests/test_gpu_axes_slab.py tests/test_gpu_axes_stream.py > $O/tests.log 2>&1 || exit 1
for lib in new before; do
  if [ $lib = before ]; then export PYAS_TREE=$R/tools/r03_pkg; else unset PYAS_TREE; fi
  timeout -k 10 300 python -u tools/bench_zeros.py --zeros 0.5 --axes none,0,2 --reps 5 > $O/zeros50_$lib.json 2> $O/zeros50_$lib.err || exit 1
  (cd /tmp && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zt_$lib -o run -- \
     python3 $R/tools/bench_zeros.py --zeros 0.5 --axes none,0,2 --reps 5 > $R/$O/zeros50_${lib}_prof.log 2>&1) || exit 1
  cp $(find /tmp/zt_$lib -name '*kernel_stats.csv' | head -n 1) $O/zeros50_${lib}_kernel_stats.csv
done
unset PYAS_TREE
timeout -k 10 300 python -u tools/bench_zeros.py --zeros 0 --axes none,0,2 --reps 5 > $O/zeros0.json 2> $O/zeros0.err || exit 1
timeout -k 10 300 python -u tools/bench_zeros.py --zeros 0.02 --axes none,0,2 --reps 5 > $O/zeros2.json 2> $O/zeros2.err || exit 1
timeout -k 10 300 python -u tools/bench_axes.py > $O/axes_plain.json 2> $O/axes_plain.err || exit 1
timeout -k 10 300 python -u tools/bench_axes.py --rec sum > $O/axes_plain_rec.json 2> $O/axes_plain_rec.err || exit 1
timeout -k 10 300 python -u tools/bench_axes.py --shuffle > $O/axes_shuf.json 2> $O/axes_shuf.err || exit 1
PYAS_SHUF_SLAB=0 timeout -k 10 300 python -u tools/bench_axes.py --shuffle --only 1 > $O/axes_shuf_noslab.json 2> $O/axes_shuf_noslab.err || exit 1
timeout -k 10 300 python -u tools/bench_axes.py --shuffle --rec sum > $O/axes_shuf_rec.json 2> $O/axes_shuf_rec.err || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_inflate.py > $O/inflate_tests.log 2>&1 || exit 1
for lib in new before; do
  if [ $lib = before ]; then export PYAS_TREE=$R/tools/r03_pkg; else unset PYAS_TREE; fi
  timeout -k 10 300 python -u tools/bench_inflate.py --sweep 1,8,30,256 > $O/inflate_bench_$lib.json 2> $O/inflate_bench_$lib.err || exit 1
done
PYAS_LIB=$R/pyactivestorage_amd/lib/before/libpyas_prof.so timeout -k 10 300 python -u tools/bench_inflate.py --chunks 64 --reps 1 --no-check > $O/inflate_phase_profile.txt 2>&1 || exit 1
