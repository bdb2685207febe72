set -o pipefail
mkdir -p gpurun_out/r02
run() { env "$@" timeout -k 10 200 python -u tools/bench_dropin.py --zlib --chunks 1024 --gpu-only --trials 2 >> gpurun_out/r02/dropin_zlib_knobs.jsonl 2>> gpurun_out/r02/dropin_zlib_knobs.err; }
run PYAS_COALESCE_DEPTH=4 || exit 2
run PYAS_COALESCE_DEPTH=1 || exit 3
run PYAS_COALESCE_ZEROCOPY=0 || exit 4
run PYAS_COALESCE_DEPTH=8 || exit 5
