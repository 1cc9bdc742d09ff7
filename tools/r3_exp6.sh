#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
bash tools/ab.sh "--no-check" cur norec
for d in 0 1 2 4 7; do
  BIC_LIB_PATH=binary-image-compression_amd/lib/libbic_stamps.so BIC_EMIT_DBG=$d timeout -k 10 120 python3 bench.py --no-cpu --no-check --steps 10 > gpurun_out/dbg_$d.log 2>&1 || { echo "dbg $d failed"; tail -5 gpurun_out/dbg_$d.log; exit 1; }
  python3 -c "
import json
l=[x for x in open('gpurun_out/dbg_$d.log') if x.startswith('{')][-1]; j=json.loads(l)
print('dbg $d', j['ms_per_step'], {k:round(v['avg_us'],1) for k,v in j['kernels'].items()})"
done
