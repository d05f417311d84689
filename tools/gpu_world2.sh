#!/bin/bash
# Multi-rank rehearsal of the driver's N>1 bench on a one-GPU box: two ranks
# share cuda:0 over gloo (RCCL admits one rank per device); checks that rank 0
# prints one JSON line with n_gpus 2 and the job totals of both ranks.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/w2
FOGNET_BENCH_SHARE_GPU=1 FOGNET_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 \
  --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29531 bench.py --gpus 2 --steps 3 --warmup 1 \
  > gpurun_out/w2/bench_world2.log 2>&1 || { tail -20 gpurun_out/w2/bench_world2.log; exit 1; }
grep '^{' gpurun_out/w2/bench_world2.log | tail -n 1 > gpurun_out/w2/bench_world2.json
python3 -c "
import json; d=json.load(open('gpurun_out/w2/bench_world2.json'))
print('n_gpus', d['n_gpus'], 'decisions', d['stats']['decisions'], 'value %.3e' % d['value'], 'ms/step', round(d['ms_per_step'],2), 'failed', d['failed_replications'])
assert d['n_gpus'] == 2 and d['stats']['decisions'] == 2 * 4096 * 100000
"
