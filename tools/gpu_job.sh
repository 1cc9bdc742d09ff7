# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -q -x --timeout 300 --timeout-method thread > gpurun_out/gpu_k1r.log 2>&1 || { tail -30 gpurun_out/gpu_k1r.log; exit 1; }
tail -2 gpurun_out/gpu_k1r.log
bash tools/ab.sh "--steps 50 --warmup 5 --workload c2" k1r0 k1r || exit 1
bash tools/ab.sh "--steps 50 --warmup 5 --workload c2" k1r0 k1r || exit 1
BIC_LIB_PATH=binary-image-compression_amd/lib/var_k1r.so timeout -k 10 180 python3 tools/c2_alt.py 2>&1 | grep -v amdgpu.ids | head -6
