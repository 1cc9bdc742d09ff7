#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py -x -q --timeout 120 --timeout-method thread -k "misaligned or encode_gray" > gpurun_out/exp10_tests.log 2>&1; rc=$?
tail -2 gpurun_out/exp10_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED|Timeout" gpurun_out/exp10_tests.log | head -20; exit 1; }
bash tools/profile_all.sh > gpurun_out/profall.log 2>&1 || { tail -5 gpurun_out/profall.log; exit 1; }
tail -1 gpurun_out/profall.log
