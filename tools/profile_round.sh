#!/bin/bash
# rocprofv3 kernel-trace stats + separate PMC passes (FETCH_SIZE, WRITE_SIZE) of one bench
# command; outputs under gpurun_out/$TAG. Usage: tools/profile_round.sh TAG [bench args...]
set -o pipefail
TAG=$1; shift
OUT=gpurun_out/$TAG
mkdir -p $OUT
export TMPDIR=/tmp
# the kernel sources this profile describes (prof_summary.py copies it into pmc_<w>.json)
python3 -c "import sys; sys.path.insert(0, 'binary-image-compression_amd'); import pybic; print(pybic.sources_hash())" > $OUT/sources.sha256
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/trace -o run --output-format csv -- python3 bench.py "$@" --no-cpu --no-check > $OUT/trace.log 2>&1 || { echo "trace failed $?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE -d $OUT/fetch -o run --output-format csv -- python3 bench.py "$@" --no-cpu --no-check > $OUT/fetch.log 2>&1 || { echo "fetch failed $?"; exit 1; }
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE -d $OUT/write -o run --output-format csv -- python3 bench.py "$@" --no-cpu --no-check > $OUT/write.log 2>&1 || { echo "write failed $?"; exit 1; }
find $OUT -name "*.csv" | head -20
