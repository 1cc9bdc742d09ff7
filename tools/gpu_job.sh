# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
for v in agew; do
BIC_LIB_PATH=binary-image-compression_amd/lib/var_$v.so timeout -k 10 600 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fullsize.py tests/test_gpu_egsrc.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6_test_$v.log 2>&1 || { tail -30 gpurun_out/r6_test_$v.log; exit 1; }
tail -1 gpurun_out/r6_test_$v.log
done
bash tools/ab.sh "--steps 20 --warmup 3" base agew agew2 agew3
