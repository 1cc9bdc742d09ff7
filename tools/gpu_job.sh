# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
bash tools/ab.sh "--steps 20 --warmup 3" cur p2 p3 p4 > gpurun_out/abx_pipe.log 2>&1 || exit 1
