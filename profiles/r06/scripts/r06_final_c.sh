# round 6 closing (c, the final binary after the strided walk and the sized LDS map):
# full GPU suite, smoke, default bench, rocprof of the c3 steps + FETCH/WRITE passes
# (profiles/traffic.json regenerated), the bench's query shapes under rocprof
set -o pipefail
O=gpurun_out/r06/final3
R=$GRAFT_REPO_ROOT
mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
bash tools/profile_config.sh c3 r06 > $O/profile_c3.log 2>&1 || exit 1
for q in "c3_slab 0" "c3_slab 4" "c3_slab 5" "c3_stride 0" "c3_stride 3" "c3_stride 4"; do
  bash $R/tools/profile_query.sh $q r06f || exit 1
done
