# round 4: the committed tree once more -- smoke, the hyperslab and golden subset, default bench, C5
set -o pipefail
O=gpurun_out/r04/check
mkdir -p $O
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "golden or select or storage or fullsize or zero_sign" > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 400 python -u bench.py --config c5 --extra none > $O/bench_c5.json 2> $O/bench_c5.err || exit 1
