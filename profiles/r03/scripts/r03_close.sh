# round-3 closing evidence: full GPU suite, smoke, default bench, rocprofv3 summaries of C3 and C5
set -o pipefail
O=gpurun_out/r03/close
mkdir -p $O
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 700 bash tools/profile_config.sh c3 r03 > $O/prof_c3.log 2>&1 || exit 1
timeout -k 10 900 bash tools/profile_config.sh c5 r03 > $O/prof_c5.log 2>&1 || exit 1
