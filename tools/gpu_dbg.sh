set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u bench.py --steps 40 --warmup 6 --inflight 2 --no-cpu > gpurun_out/if2b.log 2>&1 || exit $?
timeout -k 10 300 python -u bench.py --steps 40 --warmup 6 --no-cpu > gpurun_out/if1b.log 2>&1 || exit $?
