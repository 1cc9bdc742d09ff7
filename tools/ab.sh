#!/bin/bash
# tools/ab.sh "benchargs" NAME1 NAME2 ...: alternate bench runs over lib/var_NAME.so on one box
set -o pipefail
ARGS=$1; shift
for rep in 1 2; do
  for n in "$@"; do
    BIC_LIB_PATH=binary-image-compression_amd/lib/var_$n.so timeout -k 10 120 python3 bench.py --no-cpu $ARGS > gpurun_out/ab_$n.log 2>&1 || { echo "$n failed"; tail -5 gpurun_out/ab_$n.log; exit 1; }
    python3 -c "
import json
l=[x for x in open('gpurun_out/ab_$n.log') if x.startswith('{')][-1]; j=json.loads(l)
print('$n', j['ms_per_step'], j.get('bit_exact_check'), round(j['roofline']['avg_launch_us'],1), {k:round(v['avg_us'],1) for k,v in j['kernels'].items()})"
  done
done
