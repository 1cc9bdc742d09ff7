#!/bin/bash
# tools/ab_dec.sh NAME...: decoder kernel times over lib/var_NAME.so (rocprofv3 kernel trace of tools/run_decode.py)
set -o pipefail
export TMPDIR=/tmp
for n in "$@"; do
  BIC_LIB_PATH=binary-image-compression_amd/lib/var_$n.so timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/abdec_$n -o run --output-format csv -- python3 tools/run_decode.py > gpurun_out/abdec_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/abdec_$n.log; }
  python3 - <<PY
import csv
for r in csv.DictReader(open('gpurun_out/abdec_$n/run_kernel_stats.csv')):
    if 'dec' in r['Name'] or 'col' in r['Name']: print('$n', r['Name'][:40], r['Calls'], round(float(r['AverageNs'])/1e3,1))
PY
done
