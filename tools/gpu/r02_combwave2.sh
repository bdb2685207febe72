# wave combine (in-order butterfly + lane-0 sum chain): parity, resident A/B, trace; plane-load NT variant A/B
set -o pipefail
mkdir -p gpurun_out/r02d
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_axes_fold.py tests/test_gpu_resident.py tests/test_gpu_active.py tests/test_gpu_active_select.py tests/test_gpu_distributed_active.py > gpurun_out/r02d/tests.log 2>&1 || exit 1
for i in 1 2; do
  timeout -k 10 300 python -u tools/bench_active.py --resident --reps 30 | tail -n 1 | sed "s/^/wave /" >> gpurun_out/r02d/resident_ab.txt 2>> gpurun_out/r02d/resident.err || exit 2
  PYAS_COMBINE_WAVE=0 timeout -k 10 300 python -u tools/bench_active.py --resident --reps 30 | tail -n 1 | sed "s/^/thread /" >> gpurun_out/r02d/resident_ab.txt 2>> gpurun_out/r02d/resident.err || exit 3
done
for v in default pnt0; do
  if [ $v = default ]; then lib=""; else lib=$PWD/pyactivestorage_amd/lib/variants/libpyas_$v.so; fi
  for mode in "--fold --shuffle" "--shuffle"; do
    PYAS_LIB=$lib timeout -k 10 120 python -u tools/bench_axes.py $mode | sed "s/^/$v /" >> gpurun_out/r02d/pnt_var.txt 2>> gpurun_out/r02d/pnt_var.err || exit 4
  done
done
export TMPDIR=/tmp
root=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/cw -o run -- python3 "$root/tools/bench_active.py" --resident --reps 10 > "$root/gpurun_out/r02d/trace.log" 2>&1 || exit 5
cp "$(find /tmp/cw -name '*kernel_stats.csv' | head -n 1)" "$root/gpurun_out/r02d/resident_kernel_stats.csv"
