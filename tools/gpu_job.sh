# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
for v in ora; do
BIC_LIB_PATH=binary-image-compression_amd/lib/var_$v.so timeout -k 10 180 python3 tools/c2_alt.py 2>&1 | grep -v amdgpu.ids | head -4
done
timeout -k 10 180 python3 tools/c2_alt.py 2>&1 | grep -v amdgpu.ids | head -4
