#!/bin/bash
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fullsize.py tests/test_gpu_parity.py tests/test_gpu_decode.py -x -q --timeout 120 --timeout-method thread > gpurun_out/exp12_tests.log 2>&1; rc=$?
tail -2 gpurun_out/exp12_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED|Timeout" gpurun_out/exp12_tests.log | head -20; exit 1; }
bash tools/ab.sh "--workload c2" nosc sc
