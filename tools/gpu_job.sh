# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/gpu_full11.log 2>&1 || { tail -30 gpurun_out/gpu_full11.log; exit 1; }
tail -3 gpurun_out/gpu_full11.log
bash tools/ab.sh "--steps 20 --warmup 3" cur > gpurun_out/abx_final.log 2>&1 || exit 1
cat gpurun_out/abx_final.log
