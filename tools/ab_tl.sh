#!/bin/bash
# tools/ab_tl.sh "benchargs" FIRSTKERNEL NAME...: kernel timeline of one bench step per lib/var_NAME.so
set -o pipefail
export TMPDIR=/tmp
ARGS=$1; FK=$2; shift 2
for n in "$@"; do
  BIC_LIB_PATH=binary-image-compression_amd/lib/var_$n.so timeout -k 10 120 rocprofv3 --kernel-trace -d gpurun_out/abtl_$n -o run --output-format csv -- python3 bench.py --no-cpu --no-check --steps 10 $ARGS > gpurun_out/abtl_$n.log 2>&1 || { echo "$n failed"; tail -3 gpurun_out/abtl_$n.log; exit 1; }
  echo "== $n"; python3 tools/timeline.py gpurun_out/abtl_$n/run_kernel_trace.csv $FK
done
