# FETCH_SIZE of the lean fold on shuffled C3 chunks (plain plane loads for (1,)'s 64-B pieces)
set -o pipefail
mkdir -p gpurun_out/r02p
export TMPDIR=/tmp
root=$PWD
cd /tmp && timeout -s KILL 180 rocprofv3 --pmc FETCH_SIZE --output-format csv -d /tmp/pf -o run -- python3 "$root/tools/bench_axes.py" --fold --shuffle > "$root/gpurun_out/r02p/fetch.log" 2>&1 || exit 1
python3 - "$root" <<'PY'
import csv, glob, sys, collections
root = sys.argv[1]
f = glob.glob('/tmp/pf/**/*counter_collection.csv', recursive=True)[0]
acc = collections.defaultdict(list)
for r in csv.DictReader(open(f)):
    if 'pyas' in r['Kernel_Name']:
        acc[(r['Kernel_Name'].split('(')[0], r['Grid_Size'])].append(float(r['Counter_Value']))
with open(root + '/gpurun_out/r02p/fetch_summary.txt', 'w') as o:
    for (k, g), v in sorted(acc.items()):
        m = sum(v) / len(v)
        o.write(f"{k} grid={g} n={len(v)} FETCH_SIZE_avg={m:.0f} x2*1024/4294967296={m * 2048 / 4294967296:.4f}\n")
PY
