# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
timeout -k 10 120 python3 tools/capture_memset_probe.py > gpurun_out/cap_memset.log 2>&1 || { tail -20 gpurun_out/cap_memset.log; exit 1; }
grep "^{" gpurun_out/cap_memset.log
for e in single-kernel two-pass staged; do timeout -k 10 120 python3 tools/capture_probe.py $e > gpurun_out/cap_$e.log 2>&1 || { tail -20 gpurun_out/cap_$e.log; exit 1; }; grep replay gpurun_out/cap_$e.log | tail -1; done
timeout -k 10 600 python -u -m pytest tests/test_gpu_egsrc.py tests/test_gpu_fullsize.py tests/test_gpu_fused.py tests/test_capi.py tests/test_gpu_match.py -x -q --timeout 200 --timeout-method thread > gpurun_out/r6_test.log 2>&1 || { tail -30 gpurun_out/r6_test.log; exit 1; }
tail -2 gpurun_out/r6_test.log
bash tools/ab.sh "--steps 20 --warmup 3" base pri rlast nokmix nopri
