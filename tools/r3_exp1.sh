#!/bin/bash
# round-3 session-2 experiment: C3 kernel timeline (emission / rest overlap) + count-pass variants A/B
set -o pipefail
cd $GRAFT_REPO_ROOT
export TMPDIR=/tmp
mkdir -p gpurun_out/exp1
timeout -k 10 300 rocprofv3 --kernel-trace -d gpurun_out/exp1/trace -o run --output-format csv -- python3 bench.py --no-cpu --no-check --steps 5 --warmup 2 > gpurun_out/exp1/trace.log 2>&1 || { echo "trace failed"; exit 1; }
f=$(find gpurun_out/exp1/trace -name "*kernel_trace.csv" | head -1)
python3 tools/timeline.py $f k_gray_strips -2 > gpurun_out/exp1/timeline.txt && cat gpurun_out/exp1/timeline.txt
bash tools/ab.sh "" base gbm gpipe gbm5
