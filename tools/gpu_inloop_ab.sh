#!/bin/bash
# In-loop statistics (FOGNET_REPLAY_STATS=inloop) vs the fused epilogue (default):
# the GPU suite under the default, the statistics tests in-loop, then C3 timing of both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
FOGNET_REPLAY_STATS=inloop timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread \
  -k "stats or energy or qtime or c3_full or c4_workload or ext_lat or ring or generated" > gpurun_out/pytest_inl.log 2>&1 || { tail -30 gpurun_out/pytest_inl.log; exit 1; }
tail -2 gpurun_out/pytest_inl.log
for mode in inloop epilogue inloop epilogue; do
  FOGNET_REPLAY_STATS=$mode timeout -k 10 200 python bench.py --steps 5 --warmup 2 --no-cpu > gpurun_out/c3_$mode.log 2>&1 || exit 1
  python3 -c "
import json
l=[x for x in open('gpurun_out/c3_$mode.log') if x.startswith('{')][-1]; d=json.loads(l)
print('$mode', round(d['ms_per_step'],2), 'ms/step', round(d['roofline']['kernel_avg_ms'],2), 'kernel ms', '%.3e' % d['value'])"
done
