set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -q -x --timeout 300 --timeout-method thread tests/test_gpu_egsrc.py tests/test_gpu_fused.py tests/test_gpu_fullsize.py tests/test_gpu_multirank.py > gpurun_out/t17.log 2>&1; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python -u -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1 || exit $?
: > gpurun_out/ab17.log
for v in libbic exp_wk0 libbic exp_wk0; do
  for w in c3 c4; do
  BIC_LIB_PATH=binary-image-compression_amd/lib/$v.so timeout -k 10 240 python -u bench.py --workload $w --steps 20 --warmup 3 --no-cpu > gpurun_out/b17.json 2>> gpurun_out/ab17.err || exit $?
  python3 -c "
import json
j=json.loads([l for l in open('gpurun_out/b17.json') if l.startswith('{')][-1])
print('$v $w |', j['ms_per_step'], j.get('bit_exact_check'), {k: round(v['avg_us'],1) for k, v in j['kernels'].items()})" >> gpurun_out/ab17.log
  done
done
