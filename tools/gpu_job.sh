# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_egad.py tests/test_gpu_decode.py tests/test_gpu_fullsize.py -x -q --timeout 200 --timeout-method thread > gpurun_out/egad_t.log 2>&1 || { tail -30 gpurun_out/egad_t.log; exit 1; }
tail -1 gpurun_out/egad_t.log
timeout -k 10 200 python -u tools/time_aux.py --reps 3 > gpurun_out/egad_aux.log 2>&1 || { tail -5 gpurun_out/egad_aux.log; exit 1; }
grep '^{' gpurun_out/egad_aux.log | tail -1 | python3 -c "
import json,sys; j=json.loads(sys.stdin.read()); print({k:(v['us'] if isinstance(v,dict) else v) for k,v in j.items() if 'adaptive' in k or 'egad' in k})"
