# round 5: rocprofv3 kernel splits of single C3 query shapes (stats only kept)
O=gpurun_out/r05/qprof
R=$GRAFT_REPO_ROOT
mkdir -p $R/$O
cd /tmp && export TMPDIR=/tmp
for q in "c3_slab 0" "c3_slab 4" "c3_slab 5" "c3_stride 2" "c3_stride 1"; do
  set -- $q
  rm -rf /tmp/qp
  timeout -k 10 240 rocprofv3 --kernel-trace --stats --output-format csv -d /tmp/qp -o run -- python3 $R/tools/query_c3.py $1 $2 --reps 10 > $R/$O/${1}_$2.json 2> $R/$O/${1}_$2.err || exit 1
  cp $(find /tmp/qp -name '*kernel_stats.csv' | head -n 1) $R/$O/${1}_$2_kernel_stats.csv
done
