set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/ > gpurun_out/t21.log 2>&1 || exit $?
bash tools/profile_round.sh prof_c3 --workload c3 --steps 10 > gpurun_out/prof_c3.out 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 20 --warmup 5 > gpurun_out/final_bench3.log 2>&1 || exit $?
