#!/bin/bash
# tools/diag_ab.sh NAME...: tools/diag_time.py over lib/var_NAME.so, twice each, one JSON line per run
set -o pipefail
for rep in 1 2; do
  for n in "$@"; do
    BIC_LIB_PATH=binary-image-compression_amd/lib/var_$n.so timeout -k 10 120 python3 tools/diag_time.py 2>/dev/null || { echo "$n failed"; exit 1; }
  done
done
