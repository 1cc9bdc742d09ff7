# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
for rep in 1 2; do
for a in "" "--one-stream" "--workload c4" "--workload c4 --one-stream"; do
  timeout -k 10 200 python3 bench.py --steps 20 --warmup 3 --no-cpu $a > gpurun_out/os.log 2>&1 || { tail -5 gpurun_out/os.log; exit 1; }
  python3 -c "
import json
l=[x for x in open('gpurun_out/os.log') if x.startswith('{')][-1]; j=json.loads(l)
print('$a |', j['ms_per_step'], j.get('bit_exact_check'), {k:(v['launches'],round(v['avg_us'],1)) for k,v in j['kernels'].items()})"
done
done
