# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
BIC_LIB_PATH=binary-image-compression_amd/lib/var_both.so timeout -k 10 300 python -u -m pytest tests/test_gpu_egsrc.py tests/test_gpu_fullsize.py -q -x --timeout 200 --timeout-method thread > gpurun_out/gpu_both.log 2>&1 || { tail -30 gpurun_out/gpu_both.log; exit 1; }
tail -1 gpurun_out/gpu_both.log
bash tools/ab.sh "--steps 20 --warmup 3" base nosink ffb both || exit 1
bash tools/ab.sh "--steps 20 --warmup 3" base nosink ffb both || exit 1
