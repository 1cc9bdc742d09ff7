#!/bin/bash
# tools/dbg_first.sh N VAR...: N fresh processes per variant library lib/var_VAR.so ("default" =
# lib/libbic.so), each one first encode through tools/dbg_first.py; one JSON line per encode into
# gpurun_out/dbg_first$DBG_TAG.jsonl (DBG_ONE_STREAM=1: one stream)
set -o pipefail
N=$1; shift
out=gpurun_out/dbg_first${DBG_TAG}.jsonl
: > $out
for v in "$@"; do
  lib=binary-image-compression_amd/lib/var_$v.so
  [ "$v" = default ] && lib=binary-image-compression_amd/lib/libbic.so
  for i in $(seq 1 $N); do
    BIC_LIB_PATH=$lib timeout -k 10 120 python3 tools/dbg_first.py 70 4096 2 >> $out 2> gpurun_out/dbg_first.err || {
      echo "variant $v trial $i failed"; tail -5 gpurun_out/dbg_first.err; exit 1; }
  done
  echo "$v done"
done
