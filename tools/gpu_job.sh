# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_egsrc.py tests/test_gpu_fused.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6_test.log 2>&1 || { tail -30 gpurun_out/r6_test.log; exit 1; }
tail -2 gpurun_out/r6_test.log
for w in c3 c4; do
timeout -k 10 200 python3 bench.py --no-cpu --steps 20 --warmup 3 --workload $w > gpurun_out/b_$w.log 2>&1 || { tail -20 gpurun_out/b_$w.log; exit 1; }
python3 -c "
import json
l=[x for x in open('gpurun_out/b_$w.log') if x.startswith('{')][-1]; j=json.loads(l)
print('$w', j['ms_per_step'], j.get('bit_exact_check'), j['roofline'], {k:round(v['avg_us'],1) for k,v in j['kernels'].items()})"
done
