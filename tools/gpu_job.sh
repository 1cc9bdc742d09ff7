# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/gpu_full12.log 2>&1 || { tail -30 gpurun_out/gpu_full12.log; exit 1; }
tail -2 gpurun_out/gpu_full12.log
for w in c3 c2 c4; do
echo "== $w"
bash tools/ab.sh "--steps 20 --warmup 3 --workload $w" prev cur || exit 1
done
