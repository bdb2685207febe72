#!/bin/bash
# Collect the rocprofv3 evidence for one bench config on the GPU box:
#   1. --kernel-trace --stats (per-kernel average durations),
#   2. --pmc FETCH_SIZE and 3. --pmc WRITE_SIZE, each in its own pass
#      (MI355X_MICROARCH.md: counters in separate runs, never with traces),
# then summarise into profiles/<round>/<config>_summary.json.
# usage: tools/profile_config.sh CONFIG ROUND [extra bench args...]
set -eo pipefail
cfg=$1; rnd=$2; shift 2
root=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
out=/tmp/prof_$cfg            # raw rocprofv3 output stays off gpurun_out (size cap)
rm -rf "$out"
mkdir -p "$out" "$root/profiles/$rnd"
export TMPDIR=/tmp
save_logs() {   # on success and on failure: the bench logs, prefixed by config
    mkdir -p "$root/gpurun_out/profiles/$rnd"
    for f in "$out"/*.log; do [ -f "$f" ] && cp "$f" "$root/gpurun_out/profiles/$rnd/${cfg}_$(basename "$f")"; done
    return 0
}
trap save_logs EXIT
cd /tmp
bench=("$root/bench.py" --config "$cfg" --extra none --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 "$@")
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- \
    python3 "${bench[@]}" --steps 20 --warmup 5 > "$out/bench_trace.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- \
    python3 "${bench[@]}" --steps 4 --warmup 2 > "$out/bench_fetch.log" 2>&1
timeout -s KILL 200 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- \
    python3 "${bench[@]}" --steps 4 --warmup 2 > "$out/bench_write.log" 2>&1
stats=$(find "$out/trace" -name '*kernel_stats.csv' | head -n 1)
fetch=$(find "$out/fetch" -name '*counter_collection.csv' | head -n 1)
write=$(find "$out/write" -name '*counter_collection.csv' | head -n 1)
bytes=$(python3 -c "import json,sys; l=[x for x in open('$out/bench_trace.log') if x.startswith('{')][-1]; print(json.loads(l)['roofline']['bytes_per_launch'])")
cp "$stats" "$root/profiles/$rnd/${cfg}_kernel_stats.csv"
cp "$fetch" "$root/profiles/$rnd/${cfg}_pmc_fetch_size.csv"
cp "$write" "$root/profiles/$rnd/${cfg}_pmc_write_size.csv"
grep '^{' "$out/bench_trace.log" | tail -n 1 > "$root/profiles/$rnd/${cfg}_bench_under_rocprof.json"
python3 "$root/profiles/summarize.py" --trace "$stats" --pmc "$fetch" --pmc-write "$write" \
    --config "$cfg" --bytes "$bytes" --out "$root/profiles/$rnd/${cfg}_summary.json" \
    --traffic "$root/profiles/traffic.json"
# profiles/ is not merged back by gpurun: mirror it under gpurun_out
mkdir -p "$root/gpurun_out/profiles/$rnd"
cp "$root/profiles/$rnd/${cfg}"_* "$root/gpurun_out/profiles/$rnd/"
cp "$root/profiles/traffic.json" "$root/gpurun_out/profiles/traffic.json"
