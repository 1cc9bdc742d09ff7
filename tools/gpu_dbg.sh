set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/dbg7.log
for i in 1 2 3 4 5; do
  timeout -k 10 120 python -u tools/dbg_egsrc8.py 70 4096 1 3 >> gpurun_out/dbg7.log 2>&1 || exit $?
  BIC_LIB_PATH=binary-image-compression_amd/lib/exp_sysfence.so timeout -k 10 120 python -u tools/dbg_egsrc5.py 70 4096 1 0 0 | sed 's/^/sysfence /' >> gpurun_out/dbg7.log 2>&1 || exit $?
done
: > gpurun_out/ab7.log
for a in "--eg-source-mode 1" "--eg-source-mode 2" "--eg-source-mode 3" "--eg-source-mode 4" "--eg-source-mode 1 --one-stream" "--no-eg-source"; do
  timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu $a > gpurun_out/b7.json 2>> gpurun_out/ab7.err || exit $?
  python3 -c "
import json
j=json.loads([l for l in open('gpurun_out/b7.json') if l.startswith('{')][-1])
print('$a |', j['ms_per_step'], j.get('bit_exact_check'), {k: round(v['avg_us'],1) for k, v in j['kernels'].items()}, j['predictor_pass']['in_step'] if j.get('predictor_pass') else None)" >> gpurun_out/ab7.log
done
