# one-wave-per-output grid combine: parity, then resident box queries A/B and a kernel trace
set -o pipefail
mkdir -p gpurun_out/r02c
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_axes_fold.py tests/test_gpu_resident.py tests/test_gpu_active.py tests/test_gpu_active_select.py > gpurun_out/r02c/tests.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/bench_active.py --resident --reps 20 > gpurun_out/r02c/resident_wave.json 2> gpurun_out/r02c/resident.err || exit 2
PYAS_COMBINE_WAVE=0 timeout -k 10 300 python -u tools/bench_active.py --resident --reps 20 > gpurun_out/r02c/resident_thread.json 2>> gpurun_out/r02c/resident.err || exit 3
export TMPDIR=/tmp
root=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/cw -o run -- python3 "$root/tools/bench_active.py" --resident --reps 10 > "$root/gpurun_out/r02c/trace.log" 2>&1 || exit 4
cp "$(find /tmp/cw -name '*kernel_stats.csv' | head -n 1)" "$root/gpurun_out/r02c/resident_kernel_stats.csv"
