# round 5 closing tree (2): full GPU suite, smoke, default bench, the RCCL
# branch at world size 1, rocprofv3 of the bench's timed steps alone (the
# k_reduce average to compare with the bench line's kernel_ms_avg), and the
# slab (2,) min at 0 / 2 / 50 % zeros
set -o pipefail
O=gpurun_out/r05/final2
R=$GRAFT_REPO_ROOT
mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29543 bench.py --gpus 1 --force-dist --extra none --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 > $O/bench_torchrun_forcedist.json 2> $O/bench_torchrun_forcedist.err || exit 1
cd /tmp && export TMPDIR=/tmp && rm -rf /tmp/bp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/bp -o run -- python3 $R/bench.py --extra none --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 > $R/$O/bench_rocprof.json 2> $R/$O/bench_rocprof.err || exit 1
cp $(find /tmp/bp -name '*kernel_stats.csv' | head -n 1) $R/$O/bench_kernel_stats.csv
for z in 0 0.02 0.5; do
  rm -rf /tmp/zp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zp -o run -- python3 $R/tools/query_c3.py c3_slab 5 --method min --zeros $z --reps 10 > $R/$O/slab_min_2_z$z.json 2> $R/$O/slab_min_2_z$z.err || exit 1
  cp $(find /tmp/zp -name '*kernel_stats.csv' | head -n 1) $R/$O/slab_min_2_z${z}_kernel_stats.csv
done
