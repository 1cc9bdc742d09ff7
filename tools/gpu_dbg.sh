set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -v -x --timeout 120 --timeout-method thread tests/test_gpu_egsrc.py > gpurun_out/t19.log 2>&1 || exit $?
