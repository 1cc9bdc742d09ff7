set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_exp.sh "--steps 30 --warmup 5" s1 s128 s512 > gpurun_out/ab_sink.log 2>&1 || exit $?
