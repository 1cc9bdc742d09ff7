#!/bin/bash
# one bench line per argument set (each bit-exact-checked), appended to gpurun_out/$1.jsonl
set -o pipefail
OUT=gpurun_out/$1.jsonl; shift
: > $OUT
for a in "$@"; do
  timeout -k 10 300 python3 bench.py $a > gpurun_out/bl.log 2>&1 || { echo "failed: $a"; tail -5 gpurun_out/bl.log; exit 1; }
  grep '^{' gpurun_out/bl.log | tail -1 >> $OUT
  python3 -c "
import json
j=json.loads(open('$OUT').readlines()[-1]); print('$a |', j['ms_per_step'], j['value'], j.get('bit_exact_check'))"
done
