# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
for w in c3 c4 c2; do
  bash tools/profile_round.sh prof_$w --workload $w --steps 10 || exit 1
done
bash tools/pmc_sq.sh sq_c3 || exit 1
echo part B1 done
