#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
bash tools/ab.sh "" cur colm
for n in cur colm; do
  BIC_LIB_PATH=binary-image-compression_amd/lib/var_$n.so timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/exp5/f_$n -o run --output-format csv -- python3 bench.py --no-cpu --no-check --steps 3 --warmup 1 > gpurun_out/exp5_f_$n.log 2>&1 || { echo "pmc $n failed"; exit 1; }
  f=$(find gpurun_out/exp5/f_$n -name "*counter_collection.csv" | head -1)
  python3 - "$f" "$n" <<'PY'
import csv, sys
from collections import defaultdict
d = defaultdict(list)
for r in csv.DictReader(open(sys.argv[1])):
    d[r['Kernel_Name'][:40]].append(float(r['Counter_Value']))
for k, v in d.items():
    if 'gray' in k or 'emit' in k:
        print(sys.argv[2], k, 'FETCH_SIZE KB avg', round(sum(v) / len(v)))
PY
done
