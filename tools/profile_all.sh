#!/bin/bash
# this round's committed profiles: rocprofv3 kernel trace + FETCH/WRITE PMC passes per workload, the
# SQ issue counters for C3, the decoders' trace + SQ counters and the side kernels' trace (time_aux)
# (outputs under gpurun_out/, summarised into profiles/rNN by the host)
set -o pipefail
export TMPDIR=/tmp
for w in ${WORKLOADS:-c3 c4 c2 c5 c3f}; do
  bash tools/profile_round.sh prof_$w --workload $w --steps 10 || exit 1
done
bash tools/pmc_sq.sh sq_c3 || exit 1
bash tools/pmc_dec.sh dec > /dev/null || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/aux -o run --output-format csv -- python3 tools/time_aux.py --reps 3 > gpurun_out/aux.log 2>&1 || exit 1
echo profiles done
