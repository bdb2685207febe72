# Bench the product library and tuning variants (tools/build_variant.sh NAME FLAGS)
# on the GPU box:
#   VARIANTS="w6 w8" CONFIGS="c3 c5" TILES="0 524288" bash tools/sweep_variants.sh
# prints: config variant tile value(GB/s) ms_per_step kernel_ms frac
set -o pipefail
mkdir -p gpurun_out/sweep
for cfg in ${CONFIGS:-c3 c2 c4 c5}; do
  for v in default ${VARIANTS:-}; do
    for tile in ${TILES:-0}; do
      if [ $v = default ]; then lib=""; else lib=$PWD/pyactivestorage_amd/lib/variants/libpyas_$v.so; fi
      log=gpurun_out/sweep/${cfg}_${v}_${tile}.log
      PYAS_LIB=$lib timeout -k 10 240 python bench.py --config $cfg --steps ${STEPS:-10} --warmup 3 \
          --cpu-chunks 0 --host-inclusive 0 --file-inclusive 0 --tile-bytes $tile > $log 2>&1 || exit 1
      python3 -c "import json;l=[x for x in open('$log') if x.startswith('{')][-1];d=json.loads(l);print('$cfg','$v','$tile',d['value'],d['ms_per_step'],d['roofline']['kernel_ms_avg'],d['roofline']['frac'])"
    done
  done
done
