# round 6: full GPU suite on the tree so far, smoke, default bench, and the
# span_plan branch-form reconstruction at -O0/-O1/-O3
set -o pipefail
O=gpurun_out/r06/full1
mkdir -p $O
for o in 0 1 3; do timeout -k 10 60 tools/dbg/bin/span_plan_branch_O$o > $O/span_plan_branch_O$o.txt 2>&1; echo "rc=$?" >> $O/span_plan_branch_O$o.txt; done
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
