# c5_strong after C3/C4 in one process: freed HBM reused (default) vs never freed (PYAS_BENCH_KEEP=1)
set -o pipefail
mkdir -p gpurun_out/r02k
timeout -k 10 300 python -u bench.py --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 > gpurun_out/r02k/default.json 2> gpurun_out/r02k/err.txt || exit 1
PYAS_BENCH_KEEP=1 timeout -k 10 300 python -u bench.py --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 > gpurun_out/r02k/keep.json 2>> gpurun_out/r02k/err.txt || exit 2
timeout -k 10 300 python -u bench.py --config c5 --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 --extra none > gpurun_out/r02k/c5.json 2>> gpurun_out/r02k/err.txt || exit 3
