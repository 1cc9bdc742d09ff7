# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
BIC_LIB_PATH=binary-image-compression_amd/lib/var_cur.so timeout -k 10 180 python3 tools/dbg_twopass.py 60 > gpurun_out/dbg_twopass2.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_egad.py tests/test_gpu_decode.py -x -q --timeout 300 --timeout-method thread > gpurun_out/gpu_q14.log 2>&1 || exit 1
timeout -k 10 120 python3 tools/egad_only.py > gpurun_out/egad_only2.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_full8.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
bash tools/c2_encoders.sh > gpurun_out/c2_enc2.log 2>&1 || exit 1
