set -o pipefail
mkdir -p gpurun_out
: > gpurun_out/dbg5.log
for cfg in "70 4096 1 0 0" "70 4096 1 0 0" "130 4096 1 0 0" "70 4096 1 0 2"; do
  timeout -k 10 120 python -u tools/dbg_egsrc5.py $cfg >> gpurun_out/dbg5.log 2>&1 || exit $?
done
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_egsrc.py tests/test_gpu_decode.py > gpurun_out/t3.log 2>&1
