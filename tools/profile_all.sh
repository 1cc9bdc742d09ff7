#!/bin/bash
# this round's committed profiles: rocprofv3 kernel trace + FETCH/WRITE PMC passes per workload, and
# the SQ issue counters for C3 (outputs under gpurun_out/, summarised into profiles/r02 by the host)
set -o pipefail
export TMPDIR=/tmp
for w in c3 c4 c2 c5 c3f; do
  bash tools/profile_round.sh prof_$w --workload $w --steps 10 || exit 1
done
bash tools/pmc_sq.sh sq_c3 || exit 1
