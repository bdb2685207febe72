set -o pipefail
mkdir -p gpurun_out/r02/occ2
for v in default fw4 u8; do
  if [ $v = default ]; then lib=""; else lib=$PWD/pyactivestorage_amd/lib/variants/libpyas_$v.so; fi
  for mode in "--fold" "--fold --shuffle" ""; do
    PYAS_LIB=$lib timeout -k 10 120 python -u tools/bench_axes.py $mode >> gpurun_out/r02/occ2/$v.jsonl 2>> gpurun_out/r02/occ2/err.log || exit 1
  done
done
