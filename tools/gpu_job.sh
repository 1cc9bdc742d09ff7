# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
BIC_LIB_PATH=binary-image-compression_amd/lib/var_cur.so timeout -k 10 180 python3 tools/dbg_twopass.py 60 >> gpurun_out/dbg_twopass.log 2>&1 || exit 1
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > gpurun_out/gpu_full7.log 2>&1
rc=$?; [ $rc -gt 1 ] && exit $rc
bash tools/ab.sh "--steps 20 --warmup 3" base cur ws1 mix > gpurun_out/ab_12_c3.log 2>&1 || exit 1
bash tools/ab.sh "--workload c4 --steps 20 --warmup 3" cur ws1 > gpurun_out/ab_12_c4.log 2>&1 || exit 1
timeout -k 10 150 python3 tools/walk_stamps.py > gpurun_out/walk_st5.log 2>&1 || exit 1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/aux12 -o run --output-format csv -- python3 tools/time_aux.py --reps 3 > gpurun_out/aux12.log 2>&1 || exit 1
