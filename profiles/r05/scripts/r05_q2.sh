# round 5: mask modes for selection / cut kernels -- parity, query profiles, bench
set -o pipefail
O=gpurun_out/r05/q2
mkdir -p $O
export TMPDIR=/tmp
T="python -u -m pytest -x -q --timeout 120 --timeout-method thread"
timeout -k 10 600 $T tests/test_gpu_spans.py tests/test_gpu_axes_cuts.py tests/test_gpu_axes_slab.py tests/test_gpu_records.py tests/test_gpu_resident.py > $O/tests.log 2>&1 || exit 1
for q in "c3_slab 0" "c3_slab 4" "c3_slab 5" "c3_stride 0" "c3_stride 1" "c3_stride 2"; do
  bash tools/profile_query.sh $q r05 >> $O/qprof.log 2>&1 || exit 1
done
timeout -k 10 500 python -u bench.py --steps 10 --extra c5,c3_slab,c3_stride --extra-steps 10 --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 > $O/bench.json 2> $O/bench.err || exit 1
