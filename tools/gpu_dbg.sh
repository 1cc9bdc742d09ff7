set -o pipefail
mkdir -p gpurun_out
# a test failure (rc 1) goes on to the next step; a fault, abort or time limit ends the script
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
timeout -k 10 300 python -u tools/dbg_egsrc.py 70 4096 > gpurun_out/dbg.log 2>&1; rc=$?; ok $rc || exit $rc
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_egad.py tests/test_gpu_decode.py tests/test_gpu_match.py -k "variants or egad or adaptive or eg_adaptive" > gpurun_out/t2.log 2>&1; rc=$?; ok $rc || exit $rc
timeout -k 10 600 python -u -m pytest -q --timeout 120 --timeout-method thread tests/test_gpu_egsrc.py tests/test_gpu_fused.py > gpurun_out/t3.log 2>&1; rc=$?; ok $rc || exit $rc
exit 0
