# tools/gpu_job.sh: one GPU call of this session's A/B and diagnostic steps (edited per call)
set -o pipefail
export TMPDIR=/tmp
for w in c4 c3; do
echo "== $w"
bash tools/ab.sh "--steps 20 --warmup 3 --workload $w" cur ra || exit 1
bash tools/ab.sh "--steps 20 --warmup 3 --workload $w" cur ra || exit 1
done
