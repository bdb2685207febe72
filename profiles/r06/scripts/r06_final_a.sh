# round 6 closing (a): full GPU suite, smoke, default bench, the RCCL branch
# at world size 1, library first-call cost, rocprof of the bench's timed
# steps and the c3 FETCH/WRITE passes (profiles/traffic.json regenerated)
set -o pipefail
O=gpurun_out/r06/final
R=$GRAFT_REPO_ROOT
mkdir -p $O
timeout -k 10 1200 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || exit 1
timeout -k 10 120 python -u tools/lib_load_time.py > $O/lib_load.json 2> $O/lib_load.err || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
timeout -k 10 400 python -u -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29549 bench.py --gpus 1 --force-dist --extra none --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 > $O/bench_torchrun_forcedist.json 2> $O/bench_torchrun_forcedist.err || exit 1
bash tools/profile_config.sh c3 r06 > $O/profile_c3.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_inflate.py --sweep 1,30,256 > $O/inflate_bench.json 2> $O/inflate_bench.err || exit 1
PYAS_INFLATE_NG=2 timeout -k 10 300 python -u tools/bench_inflate.py --sweep 1,256 > $O/inflate_bench_ng2.json 2> $O/inflate_bench_ng2.err || exit 1
PYAS_LIB=$R/pyactivestorage_amd/lib/prof/libpyas_prof.so timeout -k 10 300 python -u tools/bench_inflate.py --chunks 4 --reps 1 > $O/inflate_phase.txt 2>&1 || exit 1
timeout -k 10 600 python -u tools/bench_inflate_crossover.py --reps 5 > $O/inflate_crossover.json 2> $O/inflate_crossover.err || exit 1
# zero sign on the slab's full reduction against mean (same variable)
cd /tmp
for m in mean min; do
  for z in 0.02 0.5; do
    q=0; [ $m = min ] && q=1
    timeout -k 10 240 python3 $R/tools/query_c3.py c3_slab $q --method $m --zeros $z --reps 10 > $R/$O/zs_c3_slab_full_${m}_z$z.json 2> $R/$O/zs_c3_slab_full_${m}_z$z.err || exit 1
  done
done
