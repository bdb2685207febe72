#!/bin/bash
# rocprofv3 evidence for one C3 query shape (tools/query_c3.py): kernel-trace
# stats, then FETCH_SIZE and WRITE_SIZE in passes of their own; summary to
# profiles/<round>/queries/NAME_IDX_summary.json (mirrored under gpurun_out).
# usage: tools/profile_query.sh NAME IDX ROUND
set -o pipefail
name=$1; idx=$2; rnd=$3
R=${GRAFT_REPO_ROOT:-$(cd "$(dirname "$0")/.." && pwd)}
out=/tmp/pq_${name}_$idx
rm -rf "$out"; mkdir -p "$out" "$R/gpurun_out/profiles/$rnd/queries"
cd /tmp && export TMPDIR=/tmp
q=(python3 "$R/tools/query_c3.py" "$name" "$idx")
timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d "$out/trace" -o run -- "${q[@]}" --reps 10 > "$out/q.json" 2> "$out/q.err" || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$out/fetch" -o run -- "${q[@]}" --reps 3 > /dev/null 2> "$out/f.err" || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$out/write" -o run -- "${q[@]}" --reps 3 > /dev/null 2> "$out/w.err" || exit 1
st=$(find "$out/trace" -name '*kernel_stats.csv' | head -n 1)
fe=$(find "$out/fetch" -name '*counter_collection.csv' | head -n 1)
wr=$(find "$out/write" -name '*counter_collection.csv' | head -n 1)
d="$R/gpurun_out/profiles/$rnd/queries"
cp "$st" "$d/${name}_${idx}_kernel_stats.csv"
python3 "$R/tools/query_summary.py" "$name" "$idx" "$st" "$fe" "$wr" "$out/q.json" "$d/${name}_${idx}_summary.json"
