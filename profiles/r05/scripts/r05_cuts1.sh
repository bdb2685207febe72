# round 5: run_spans + dense cut chunks -- parity first, then the C3 query shapes
set -o pipefail
O=gpurun_out/r05/cuts1
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_spans.py tests/test_gpu_sharded.py tests/test_gpu_axes_cuts.py tests/test_gpu_axes_slab.py tests/test_gpu_records.py > $O/new_tests.log 2>&1 || exit 1
timeout -k 10 900 $T tests -m gpu -k "golden or select or storage or hyperslab or chained or coalesc or reduce_chunk or axes or active" > $O/tests.log 2>&1 || exit 1
timeout -k 10 500 python -u bench.py --extra c5,c3_slab,c3_stride --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 > $O/bench.json 2> $O/bench.err || exit 1
