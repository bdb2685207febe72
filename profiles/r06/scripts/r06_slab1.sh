# round 6: LDS-row cut kernel fast path (box spanning the run) -- cut/zero-sign
# tests, then the default bench with its c3_slab / c3_stride extras
set -o pipefail
O=gpurun_out/r06/slab1
mkdir -p $O
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_axes_cuts.py tests/test_gpu_zero_sign.py tests/test_gpu_axes_rowlds.py tests/test_gpu_axes_slab.py tests/test_gpu_records.py tests/test_gpu_spans.py > $O/tests.log 2>&1 || exit 1
timeout -k 10 400 python -u bench.py > $O/bench.json 2> $O/bench.err || exit 1
