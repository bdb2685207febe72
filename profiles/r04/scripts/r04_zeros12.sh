# round 4: lean-fold zero tracking as compare + select of the sign word; same-box mean vs min
set -o pipefail
O=gpurun_out/r04/zeros12
mkdir -p $O
export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
T="python -u -m pytest -x -q --timeout 300 --timeout-method thread"
timeout -k 10 900 $T tests/test_gpu_zero_sign.py tests/test_gpu_axes_fold.py > $O/tests.log 2>&1 || exit 1
cd /tmp
for spec in "mean:0.5" "min:0.5" "min:0"; do
  m=${spec%%:*}; z=${spec#*:}
  rm -rf /tmp/zt && timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/zt -o run -- \
     python3 $R/tools/bench_zeros.py --method $m --zeros $z --axes none,0,2 --reps 5 > $R/$O/${m}_$z.log 2>&1 || exit 1
  cp $(find /tmp/zt -name '*kernel_stats.csv' | head -n 1) $R/$O/${m}_${z}_kernel_stats.csv
done
