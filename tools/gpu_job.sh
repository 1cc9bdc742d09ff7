# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
run() {  # name, env..., bench args
  local n=$1; shift
  env "$@" timeout -k 10 120 python3 bench.py --no-cpu --steps 20 --warmup 3 > gpurun_out/bb_$n.log 2>&1 || { tail -5 gpurun_out/bb_$n.log; return 1; }
  python3 -c "
import json
l=[x for x in open('gpurun_out/bb_$n.log') if x.startswith('{')][-1]; j=json.loads(l)
print('$n', j['ms_per_step'], j.get('bit_exact_check'), round(j['roofline']['avg_launch_us'],1), {k:(v['launches'],round(v['avg_us'],1)) for k,v in j['kernels'].items()})"
}
for rep in 1 2; do
run o0p0 BIC_BAND_ORDER=0 BIC_BAND_PRIO=0 || exit 1
run o0p1 BIC_BAND_ORDER=0 BIC_BAND_PRIO=1 || exit 1
run o1p0 BIC_BAND_ORDER=1 BIC_BAND_PRIO=0 || exit 1
run o1p1 BIC_BAND_ORDER=1 BIC_BAND_PRIO=1 || exit 1
run o1p2 BIC_BAND_ORDER=1 BIC_BAND_PRIO=2 || exit 1
done
