# round 4 final tree: full GPU suite, smoke, default bench, the RCCL branch at
# world size 1 under torchrun, then the rocprofv3 summaries of the headline
# configs (kernel trace + FETCH_SIZE + WRITE_SIZE passes) into profiles/r04
set -o pipefail
O=gpurun_out/r04/final
mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --force-dist --extra none --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 > $O/bench_torchrun_forcedist.json 2> $O/bench_torchrun_forcedist.err || exit 1
timeout -k 10 700 bash tools/profile_config.sh c3 r04 > $O/prof_c3.log 2>&1 || exit 1
timeout -k 10 700 bash tools/profile_config.sh c4 r04 > $O/prof_c4.log 2>&1 || exit 1
timeout -k 10 900 bash tools/profile_config.sh c5 r04 > $O/prof_c5.log 2>&1 || exit 1
