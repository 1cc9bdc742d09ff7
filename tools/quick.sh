#!/bin/bash
# quick GPU check: staged-encoder parity tests, then the default bench line
set -o pipefail
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread -k "${QK:-fused or c3 or c4}" > gpurun_out/quick_test.log 2>&1 || { tail -30 gpurun_out/quick_test.log; exit 1; }
tail -2 gpurun_out/quick_test.log
timeout -k 10 200 python bench.py --no-cpu "$@" > gpurun_out/quick_bench.log 2>&1 || { tail -20 gpurun_out/quick_bench.log; exit 1; }
python3 -c "
import json
l=[x for x in open('gpurun_out/quick_bench.log') if x.startswith('{')][-1]; j=json.loads(l)
print(j['ms_per_step'], j.get('bit_exact_check'), j['roofline']['avg_launch_us'], j['roofline']['frac'], {k:round(v['avg_us'],1) for k,v in j['kernels'].items()})"
