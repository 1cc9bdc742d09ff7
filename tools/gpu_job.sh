# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
bash tools/ab.sh "--steps 20 --warmup 3" base o4 o4p1 o4p3 || exit 1
bash tools/ab.sh "--steps 20 --warmup 3 --workload c4" base o4p1 o4p3
