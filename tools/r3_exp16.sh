#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread -k "gray or c3 or p5 or round_trip" > gpurun_out/exp16_tests.log 2>&1; rc=$?
tail -2 gpurun_out/exp16_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED|Timeout" gpurun_out/exp16_tests.log | head -20; exit 1; }
bash tools/ab.sh "--store-planes" w4 spn
bash tools/ab.sh "" w4 spn
