# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/stamps_c2b.py > gpurun_out/stamps_c2b.log 2>&1 || { tail -20 gpurun_out/stamps_c2b.log; exit 1; }
grep -v "amdgpu.ids\|   row " gpurun_out/stamps_c2b.log
