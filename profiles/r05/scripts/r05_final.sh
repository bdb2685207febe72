# round 5 closing tree: full GPU suite, smoke, default bench, the RCCL branch at world size 1
set -o pipefail
O=gpurun_out/r05/final
mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541 bench.py --gpus 1 --force-dist --extra none --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 > $O/bench_torchrun_forcedist.json 2> $O/bench_torchrun_forcedist.err || exit 1
# the default bench under rocprofv3: the dominant kernel's stats (profiles/r05/final)
cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/bp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/bp -o run -- python3 $GRAFT_REPO_ROOT/bench.py --extra none > $GRAFT_REPO_ROOT/$O/bench_rocprof.json 2> $GRAFT_REPO_ROOT/$O/bench_rocprof.err || exit 1
cp $(find /tmp/bp -name '*kernel_stats.csv' | head -n 1) $GRAFT_REPO_ROOT/$O/bench_kernel_stats.csv
