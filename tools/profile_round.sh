#!/bin/bash
# rocprofv3 kernel-trace stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of one bench
# command; outputs under gpurun_out/$TAG. Usage: tools/profile_round.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py "$@" --no-cpu --no-check > $OUT/trace.log 2>&1 || { echo "trace failed $?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py "$@" --no-cpu --no-check > $OUT/fetch.log 2>&1 || { echo "fetch failed $?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py "$@" --no-cpu --no-check > $OUT/write.log 2>&1 || { echo "write failed $?"; exit 1; }
find $OUT -name "*.csv" | head -20
