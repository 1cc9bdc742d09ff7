# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
bash tools/ab.sh "--workload c4 --steps 20 --warmup 3" cur kb2 kb3 > gpurun_out/ab_kb.log 2>&1 || exit 1
