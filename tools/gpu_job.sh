# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/egad_prof -o run --output-format csv -- python3 tools/egad_only.py > gpurun_out/egad_prof.log 2>&1 || { tail -5 gpurun_out/egad_prof.log; exit 1; }
grep '^{' gpurun_out/egad_prof.log | tail -2
