#!/bin/bash
# Multi-rank rehearsal of the driver's N>1 bench on a one-GPU box: two ranks
# share cuda:0 over gloo (RCCL admits one rank per device); checks that rank 0
# prints one JSON line with n_gpus 2 and the job totals of both ranks.
# WORKLOADS (default "c3"): any of c3 c5 c5_REF_V3 c4 c1, one torchrun each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/w2
port=29531
for w in ${WORKLOADS:-c3}; do
  case $w in
    c3) args="--steps 3 --warmup 1"; want="2 * 4096 * 100000" ;;
    c5) args="--workload c5 --steps 3 --warmup 1 --no-cpu"; want="1024 * 10000" ;;
    c5_REF_V3) args="--workload c5 --policy REF_V3 --steps 3 --warmup 1 --no-cpu"; want="1024 * 10000" ;;
    c4) args="--workload c4 --steps 1 --warmup 1 --no-cpu"; want=None ;;
    c1) args="--workload c1 --steps 1 --warmup 1 --no-cpu"; want=None ;;
    *) echo "unknown workload $w"; exit 2 ;;
  esac
  echo "== world2 $w $(date +%T)"
  FOGNET_BENCH_SHARE_GPU=1 FOGNET_BENCH_BACKEND=gloo timeout -k 10 500 python -m torch.distributed.run --nnodes=1 \
    --nproc-per-node 2 --master-addr 127.0.0.1 --master-port $port bench.py --gpus 2 $args \
    > gpurun_out/w2/bench_world2_$w.log 2>&1 || { tail -20 gpurun_out/w2/bench_world2_$w.log; exit 1; }
  port=$((port + 1))
  grep '^{' gpurun_out/w2/bench_world2_$w.log | tail -n 1 > gpurun_out/w2/bench_world2_$w.json
  python3 -c "
import json; d=json.load(open('gpurun_out/w2/bench_world2_$w.json'))
st=d.get('stats', {})
print('$w', 'n_gpus', d['n_gpus'], 'decisions', st.get('decisions'), 'value %.3e' % d['value'], 'ms/step', round(d['ms_per_step'],2), 'failed', d.get('failed_replications'))
assert d['n_gpus'] == 2 and not d.get('failed_replications')
want = $want
assert want is None or st.get('decisions') == want, (st.get('decisions'), want)
" || exit 1
done
