#!/bin/bash
# side images (walk encodes the mixed-k rows; no k_emit_rest / fork / join): parity, then A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_fused.py tests/test_gpu_fullsize.py -x -q --timeout 120 --timeout-method thread > gpurun_out/exp2_tests.log 2>&1; rc=$?
tail -3 gpurun_out/exp2_tests.log
[ $rc -ne 0 ] && { grep -E "Error|assert|FAILED" gpurun_out/exp2_tests.log | head -20; exit 1; }
bash tools/ab.sh "" base side sideonly gbm
bash tools/ab.sh "--workload c4" base side
