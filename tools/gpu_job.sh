# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
: > gpurun_out/repeat_lines.jsonl
for a in "" "" "" "" "" "--workload c2 --steps 50" "--workload c2 --steps 50" "--workload c4" "--workload c4" "--workload c3f"; do
  timeout -k 10 300 python3 bench.py --steps 20 --warmup 5 --no-cpu $a > gpurun_out/rl.log 2>&1 || { tail -5 gpurun_out/rl.log; exit 1; }
  grep '^{' gpurun_out/rl.log | tail -1 >> gpurun_out/repeat_lines.jsonl
  python3 -c "
import json
j=json.loads(open('gpurun_out/repeat_lines.jsonl').readlines()[-1]); print('$a |', j['ms_per_step'], j.get('bit_exact_check'), j['roofline']['frac'], j['roofline']['traffic'])"
done
