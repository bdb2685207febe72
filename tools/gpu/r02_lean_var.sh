# lean column fold tuning variants (tools/build_variant_part3.sh): fold parity on the default, then C3 fold throughput
set -o pipefail
mkdir -p gpurun_out/r02
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_axes_fold.py > gpurun_out/r02/lean_tests.log 2>&1 || exit 1
for v in default d5 d3w5 d2reg; do
  if [ $v = default ]; then lib=""; else lib=$PWD/pyactivestorage_amd/lib/variants/libpyas_$v.so; fi
  for mode in "--fold" "--fold --shuffle"; do
    PYAS_LIB=$lib timeout -k 10 120 python -u tools/bench_axes.py $mode | sed "s/^/$v /" >> gpurun_out/r02/lean_var.txt 2>> gpurun_out/r02/lean_var.err || exit 2
  done
done
