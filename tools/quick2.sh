#!/bin/bash
# GPU check of the staged encoder: parity tests (fused + fullsize), then bench lines (default and extra args)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/q2_test.log 2>&1 || { tail -30 gpurun_out/q2_test.log; exit 1; }
tail -2 gpurun_out/q2_test.log
i=0
for a in "$@"; do
  i=$((i+1))
  timeout -k 10 200 python bench.py --no-cpu $a > gpurun_out/q2_b$i.log 2>&1 || { tail -20 gpurun_out/q2_b$i.log; exit 1; }
  python3 -c "
import json
l=[x for x in open('gpurun_out/q2_b$i.log') if x.startswith('{')][-1]; j=json.loads(l)
print('$a |', j['ms_per_step'], j.get('bit_exact_check'), j['roofline']['avg_launch_us'] if j['roofline'] else None, {k:round(v['avg_us'],1) for k,v in j['kernels'].items()})"
done
