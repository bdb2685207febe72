# occupancy-floor variants of the partial-axis kernels (tools/build_variant.sh)
set -o pipefail
mkdir -p gpurun_out/r02/occ
for v in default vA vB vC; do
  if [ $v = default ]; then lib=""; else lib=$PWD/pyactivestorage_amd/lib/variants/libpyas_$v.so; fi
  for mode in "" "--fold" "--shuffle" "--fold --shuffle"; do
    PYAS_LIB=$lib timeout -k 10 120 python -u tools/bench_axes.py $mode >> gpurun_out/r02/occ/$v.jsonl 2>> gpurun_out/r02/occ/err.log || exit 1
  done
done
