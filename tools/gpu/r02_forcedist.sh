# RCCL branch of bench.py at world size 1 (torchrun), and the launcher's refusal of --gpus 2 on a 1-GPU box
set -o pipefail
mkdir -p gpurun_out/r02fd
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29512 bench.py --gpus 1 --force-dist --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 > gpurun_out/r02fd/bench_forcedist.json 2> gpurun_out/r02fd/bench_forcedist.err || exit 1
timeout -k 10 60 python bench.py --gpus 2 > gpurun_out/r02fd/bench_gpus2.out 2>&1; echo "gpus2 rc=$?" >> gpurun_out/r02fd/bench_gpus2.out
exit 0
