# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
export BIC_VERBOSE=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_prof.py tests/test_gpu_multirank.py -x -q --timeout 200 --timeout-method thread > gpurun_out/dbg_t.log 2>&1; rc=$?; tail -15 gpurun_out/dbg_t.log; exit $rc
