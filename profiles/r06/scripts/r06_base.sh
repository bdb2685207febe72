# round 6 start: the restored tree on a fresh box -- full GPU suite, smoke,
# default bench, and the inflate rates (2048 x 1 MiB, per-stream sweep) the
# round's inflate work starts from
set -o pipefail
O=gpurun_out/r06/base
mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 300 python -u tools/bench_inflate.py --sweep 1,8,30,256 > $O/inflate.json 2> $O/inflate.err || exit 1
