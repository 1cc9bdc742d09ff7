set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_egsrc.py tests/test_gpu_decode.py > gpurun_out/t13.log 2>&1; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
: > gpurun_out/ab13.log
for v in libbic exp_nt libbic exp_nt; do
  BIC_LIB_PATH=binary-image-compression_amd/lib/$v.so timeout -k 10 240 python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/b13.json 2>> gpurun_out/ab13.err || exit $?
  python3 -c "
import json
j=json.loads([l for l in open('gpurun_out/b13.json') if l.startswith('{')][-1])
print('$v |', j['ms_per_step'], j.get('bit_exact_check'), {k: round(v['avg_us'],1) for k, v in j['kernels'].items()})" >> gpurun_out/ab13.log
done
bash tools/bench_lines.sh r04lines "--steps 20 --warmup 5" "--workload c2 --steps 50 --no-cpu" "--workload c3f --steps 20 --no-cpu" "--workload c4 --steps 20 --no-cpu" "--workload c5 --steps 50 --no-cpu" "--workload c1 --steps 5 --no-cpu" "--workload c1m --steps 5 --no-cpu" "--store-planes --steps 20 --no-cpu" > gpurun_out/lines.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/time_aux.py --reps 3 > gpurun_out/time_aux.json 2> gpurun_out/time_aux.err || exit 1
