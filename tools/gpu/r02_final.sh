# round-2 closing check: full GPU suite, smoke, default bench, fold A/B numbers, drop-in
set -o pipefail
mkdir -p gpurun_out/r02z
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/r02z/gpu_tests.log 2>&1 || exit 1
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > gpurun_out/r02z/smoke.log 2>&1 || exit 2
timeout -k 10 300 python -u bench.py > gpurun_out/r02z/bench_default.json 2> gpurun_out/r02z/bench_default.err || exit 3
for mode in "--fold" "--fold --shuffle" "" "--shuffle"; do
  timeout -k 10 120 python -u tools/bench_axes.py $mode >> gpurun_out/r02z/axes.jsonl 2>> gpurun_out/r02z/axes.err || exit 4
done
timeout -k 10 300 python -u tools/bench_active.py --resident --reps 30 > gpurun_out/r02z/resident.json 2> gpurun_out/r02z/resident.err || exit 5
timeout -k 10 300 python -u tools/bench_dropin.py --chunks 4096 --trials 3 --ceiling-read > gpurun_out/r02z/dropin_bench.json 2> gpurun_out/r02z/dropin_bench.err || exit 6
export TMPDIR=/tmp
root=$PWD
cd /tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/fz -o run -- python3 "$root/tools/bench_axes.py" --fold --shuffle > "$root/gpurun_out/r02z/trace_foldshuf.log" 2>&1 || exit 7
cp "$(find /tmp/fz -name '*kernel_stats.csv' | head -n 1)" "$root/gpurun_out/r02z/foldshuffle_kernel_stats.csv"
