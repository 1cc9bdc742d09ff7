# round-end evidence, part A: the GPU suite, the default bench line and one bench line per workload
# (outputs under gpurun_out/; summarised into profiles/rNN on the host). Part B: tools/profile_all.sh
set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/final_tests.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/final_bench.log 2>&1 || exit $?
bash tools/bench_lines.sh final_lines "--workload c2 --steps 50" "--workload c3f --steps 20" \
  "--workload c4 --steps 20" "--workload c5 --steps 20" "--workload c1" "--workload c1m" "--store-planes --steps 20" \
  "--inflight 2 --steps 40" > gpurun_out/final_lines.log 2>&1 || exit $?
