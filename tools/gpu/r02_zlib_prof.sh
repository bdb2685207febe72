# Active zlib query: host profile + kernel/copy timeline
set -o pipefail
mkdir -p gpurun_out/r02z
timeout -k 10 300 python -u tools/bench_active.py --zlib --axes none --reps 3 --profile > gpurun_out/r02z/active_zlib_profile.txt 2>&1 || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --memory-copy-trace --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r02z/trace -o run -- python3 $GRAFT_REPO_ROOT/tools/bench_active.py --zlib --axes none --reps 1 > $GRAFT_REPO_ROOT/gpurun_out/r02z/trace.log 2>&1 || exit 2
