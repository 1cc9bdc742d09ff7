set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
bash tools/ab_exp.sh "--steps 30 --warmup 5" base b22 wpe4 k1b2 > gpurun_out/ab_k3.log 2>&1 || exit $?
