set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py > gpurun_out/final_bench4.log 2>&1 || exit $?
for w in c4 c2 c5 c3f; do bash tools/profile_round.sh prof_$w --workload $w --steps 10 > gpurun_out/prof_$w.out 2>&1 || exit $?; done
