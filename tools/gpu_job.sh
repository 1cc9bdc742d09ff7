# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
BIC_LIB_PATH=binary-image-compression_amd/lib/var_eg3.so timeout -k 10 600 python -u -m pytest tests/test_gpu_egad.py tests/test_gpu_decode.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_q18.log 2>&1 || exit 1
for v in cur dec2 eg3 cur dec2 eg3; do BIC_LIB_PATH=binary-image-compression_amd/lib/var_$v.so timeout -k 10 120 python3 tools/egad_only.py 2>/dev/null | sed "s/^/$v /" >> gpurun_out/egad_ab18.log || exit 1; done
