# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_full9.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
timeout -k 10 120 python3 tools/egad_only.py > gpurun_out/egad_only4.log 2>&1 || exit 1
bash tools/ab.sh "--steps 20 --warmup 3" cur > gpurun_out/ab_16_c3.log 2>&1 || exit 1
