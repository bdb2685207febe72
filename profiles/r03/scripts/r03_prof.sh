# round-3 rocprofv3 summaries of the headline configs (kernel trace + FETCH_SIZE + WRITE_SIZE passes)
set -o pipefail
O=gpurun_out/r03/close
mkdir -p $O
timeout -k 10 700 bash tools/profile_config.sh c3 r03 > $O/prof_c3.log 2>&1 || exit 1
timeout -k 10 700 bash tools/profile_config.sh c4 r03 > $O/prof_c4.log 2>&1 || exit 1
timeout -k 10 900 bash tools/profile_config.sh c5 r03 > $O/prof_c5.log 2>&1 || exit 1
