set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 400 python -u tools/bench_active.py --resident --reps 10 --profile > gpurun_out/r02/active_resident_prof.log 2>&1 || exit 1
