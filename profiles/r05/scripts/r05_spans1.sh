# round 5: run_spans (predicate stream of cut chunks) -- parity, then the hyperslab rates
set -o pipefail
O=gpurun_out/r05/spans1
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 300 $T tests/test_gpu_spans.py tests/test_gpu_sharded.py > $O/spans_tests.log 2>&1 || exit 1
timeout -k 10 900 $T tests -m gpu -k "golden or select or storage or fullsize or hyperslab or chained or coalesc or reduce_chunk" > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py --extra c5,c3_slab,c3_stride --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 > $O/bench.json 2> $O/bench.err || exit 1
