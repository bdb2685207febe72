# closing rocprofv3 evidence with the final library: C3 (headline) and C5, trace + FETCH + WRITE passes
set -o pipefail
mkdir -p gpurun_out/profiles/r02
for cfg in c3 c5; do
  bash tools/profile_config.sh $cfg r02 --extra none > gpurun_out/profiles/r02/${cfg}_profile.log 2>&1 || exit 1
done
