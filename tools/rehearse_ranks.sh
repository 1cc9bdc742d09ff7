#!/bin/bash
# Functional rehearsal of bench.py's N-rank paths on ONE GPU: 2 ranks over gloo sharing cuda:0
# (BIC_BENCH_BACKEND=gloo). Times are not scaling numbers (both ranks share one device); the
# lines show the launcher, barriers, max-over-ranks timing and the stream gathers run end to end.
set -o pipefail
export BIC_BENCH_BACKEND=gloo MASTER_ADDR=127.0.0.1
OUT=gpurun_out/rehearsal_2rank.jsonl
: > $OUT
for args in "--workload c3" "--workload c3 --shard planes" "--workload c4" "--workload c5"; do
  timeout -k 10 240 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
    --master-port 29512 bench.py --gpus 2 --steps 5 --warmup 2 --no-cpu $args > gpurun_out/reh.log 2>&1 \
    || { echo "failed: $args"; tail -20 gpurun_out/reh.log; exit 1; }
  grep '^{' gpurun_out/reh.log | tail -1 >> $OUT
done
python3 -c "
import json
for l in open('$OUT'):
    j=json.loads(l); print(j['n_gpus'], j['config']['workload'][:50], j['config']['parallelism'], j['ms_per_step'], j['bit_exact_check'], j['scaling'])"
