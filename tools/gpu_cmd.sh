set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_egsrc.py tests/test_gpu_fused.py tests/test_gpu_match.py -k "egsrc or eg_source or gray or variants" > gpurun_out/t1.log 2>&1 && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu > gpurun_out/b1.json 2> gpurun_out/b1.err && \
timeout -k 10 300 python -u bench.py --steps 20 --warmup 3 --no-cpu --no-eg-source > gpurun_out/b1_old.json 2>> gpurun_out/b1.err
