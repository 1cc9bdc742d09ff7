set -o pipefail
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest -q -x --timeout 120 --timeout-method thread tests/test_gpu_egad.py tests/test_gpu_decode.py tests/test_gpu_fused.py tests/test_gpu_egsrc.py > gpurun_out/t14.log 2>&1; rc=$?
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
bash tools/bench_lines.sh r04c4 "--workload c4 --steps 20 --no-cpu" "--workload c2 --steps 50 --no-cpu" "--workload c2 --steps 50 --no-cpu --encoder staged" "--steps 20 --no-cpu" "--shard planes --plane-count 1 --steps 20 --no-cpu" "--shard planes --plane-count 2 --steps 20 --no-cpu" "--shard planes --plane-count 4 --steps 20 --no-cpu" > gpurun_out/lines14.log 2>&1 || exit 1
timeout -k 10 300 python -u tools/time_aux.py --reps 3 > gpurun_out/time_aux14.json 2> gpurun_out/time_aux.err || exit 1
