set -o pipefail
for e in auto staged two-pass; do
  BIC_LIB_PATH=binary-image-compression_amd/lib/var_cur.so timeout -k 10 120 python3 bench.py --no-cpu --workload c2 --steps 50 --warmup 5 --encoder $e > gpurun_out/c2_$e.log 2>&1 || { echo "$e failed"; tail -5 gpurun_out/c2_$e.log; exit 1; }
  python3 -c "
import json
l=[x for x in open('gpurun_out/c2_$e.log') if x.startswith('{')][-1]; j=json.loads(l)
print('$e', j['ms_per_step'], j.get('bit_exact_check'), {k:round(v['avg_us'],1) for k,v in j['kernels'].items()})"
done
