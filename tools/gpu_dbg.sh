set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python -u tools/dbg_egsrc9.py 130 4096 smooth > gpurun_out/dbg9.log 2>&1 || exit $?
timeout -k 10 200 python -u tools/dbg_egsrc9.py 70 4096 uniform >> gpurun_out/dbg9.log 2>&1 || exit $?
timeout -k 10 300 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_egsrc.py > gpurun_out/t9.log 2>&1; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
: > gpurun_out/ab9.log
for a in "--eg-source-mode 1" "--eg-source-mode 1 --one-stream"; do
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu $a > gpurun_out/b9.json 2>> gpurun_out/ab9.err || exit $?
  python3 -c "
import json
j=json.loads([l for l in open('gpurun_out/b9.json') if l.startswith('{')][-1])
print('$a |', j['ms_per_step'], j.get('bit_exact_check'), {k: round(v['avg_us'],1) for k, v in j['kernels'].items()})" >> gpurun_out/ab9.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof9 -o run --output-format csv -- python3 bench.py --steps 10 --no-cpu --no-check --one-stream > gpurun_out/prof9.log 2>&1
