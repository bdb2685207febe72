# default bench (extras now warm up like the headline): twice
set -o pipefail
mkdir -p gpurun_out/r02b
timeout -k 10 300 python -u bench.py > gpurun_out/r02b/bench1.json 2> gpurun_out/r02b/bench1.err || exit 1
timeout -k 10 300 python -u bench.py > gpurun_out/r02b/bench2.json 2> gpurun_out/r02b/bench2.err || exit 2
