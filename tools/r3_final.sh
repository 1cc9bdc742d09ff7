#!/bin/bash
# round-3 end: full GPU suite, smoke, bench lines of every workload (bit-exact, CPU baselines beside them)
set -o pipefail
cd $GRAFT_REPO_ROOT
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_tests.log 2>&1 || { tail -30 gpurun_out/final_tests.log; exit 1; }
tail -2 gpurun_out/final_tests.log
timeout -k 10 120 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 || { tail -5 gpurun_out/final_smoke.log; exit 1; }
tail -1 gpurun_out/final_smoke.log
bash tools/bench_lines.sh final_lines "" "--workload c2" "--workload c5" "--workload c3f" "--workload c4" "--workload c1m" "--workload c1" || exit 1
bash tools/bench_lines.sh final_planes "--shard planes --plane-count 1 --no-cpu" "--shard planes --plane-count 2 --no-cpu" "--shard planes --plane-count 4 --no-cpu" "--shard planes --plane-count 8 --no-cpu" || exit 1
