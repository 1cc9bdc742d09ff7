# tools/gpu_job2.sh: the second half of this round's profiles (C5, c3f, the decoders, the side kernels)
set -o pipefail
export TMPDIR=/tmp
for w in c5 c3f; do
  bash tools/profile_round.sh prof_$w --workload $w --steps 10 || exit 1
done
bash tools/pmc_dec.sh dec > /dev/null || exit 1
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/aux -o run --output-format csv -- python3 tools/time_aux.py --reps 3 > gpurun_out/aux.log 2>&1 || exit 1
echo part B2 done
