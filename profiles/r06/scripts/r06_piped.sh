# round 6: piped partial-axis box queries (result copy overlapped with the
# next slab's reduction) and k_reduce_axes with an LDS offset map sized to the
# chunk: GPU tests, the c3_slab / c3_stride extras piped and unpiped, rocprof
set -o pipefail
O=gpurun_out/r06/piped
R=$GRAFT_REPO_ROOT
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
    -k "piped or axes or active or golden or records or spans or zero_sign or resident" > $O/gpu_tests.log 2>&1 || exit 1
B="--extra c3_slab,c3_stride --steps 3 --warmup 1 --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0"
timeout -k 10 400 python -u bench.py $B > $O/bench_piped.json 2> $O/bench_piped.err || exit 1
PYAS_PIPE_SLABS=1 timeout -k 10 400 python -u bench.py $B > $O/bench_unpiped.json 2> $O/bench_unpiped.err || exit 1
for q in "c3_stride 3" "c3_stride 4" "c3_slab 4" "c3_slab 5"; do
  bash $R/tools/profile_query.sh $q r06p || exit 1
done
