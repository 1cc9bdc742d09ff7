# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fullsize.py tests/test_gpu_decode.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6_test.log 2>&1 || { tail -30 gpurun_out/r6_test.log; exit 1; }
tail -2 gpurun_out/r6_test.log
bash tools/ab.sh "--steps 20 --warmup 3 --workload c4" nomix mix mixw7
