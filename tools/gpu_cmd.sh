set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/t_all.log 2>&1; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
: > gpurun_out/ab8.log
for a in "--eg-source-mode 1" "--eg-source-mode 2" "--eg-source-mode 1 --one-stream"; do
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu $a > gpurun_out/b8.json 2>> gpurun_out/ab8.err || exit $?
  python3 -c "
import json
j=json.loads([l for l in open('gpurun_out/b8.json') if l.startswith('{')][-1])
print('$a |', j['ms_per_step'], j.get('bit_exact_check'), {k: round(v['avg_us'],1) for k, v in j['kernels'].items()}, j['predictor_pass']['in_step']['frac'] if j.get('predictor_pass') else None)" >> gpurun_out/ab8.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof8 -o run --output-format csv -- python3 bench.py --steps 10 --no-cpu --no-check > gpurun_out/prof8.log 2>&1
