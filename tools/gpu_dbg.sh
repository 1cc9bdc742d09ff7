set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_egsrc.py > gpurun_out/t11.log 2>&1; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
: > gpurun_out/ab11.log
for v in libbic exp_b21 exp_b82 exp_b43 libbic; do
  BIC_LIB_PATH=binary-image-compression_amd/lib/$v.so timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/b11.json 2>> gpurun_out/ab11.err || exit $?
  python3 -c "
import json
j=json.loads([l for l in open('gpurun_out/b11.json') if l.startswith('{')][-1])
print('$v |', j['ms_per_step'], j.get('bit_exact_check'), {k: round(v['avg_us'],1) for k, v in j['kernels'].items()})" >> gpurun_out/ab11.log
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof11 -o run --output-format csv -- python3 bench.py --steps 10 --no-cpu --no-check --one-stream > gpurun_out/prof11.log 2>&1
