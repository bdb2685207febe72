# lean column fold tuning variants (tools/build_variant_part3.sh): C3 fold throughput
set -o pipefail
mkdir -p gpurun_out/r02
for v in default r0d1w5 r1d2 r1d1w5; do
  if [ $v = default ]; then lib=""; else lib=$PWD/pyactivestorage_amd/lib/variants/libpyas_$v.so; fi
  for mode in "--fold" "--fold --shuffle"; do
    PYAS_LIB=$lib timeout -k 10 120 python -u tools/bench_axes.py $mode | sed "s/^/$v /" >> gpurun_out/r02/lean_var.txt 2>> gpurun_out/r02/lean_var.err || exit 1
  done
done
