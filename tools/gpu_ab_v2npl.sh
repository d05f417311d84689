#!/bin/bash
# v2 replay_v2_kernel<NPL>: batched firings (in-tree library) -- the v2 GPU tests, then
# per-step time at wider node sets against the one-event-per-step build (build/live/v2nobatch).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/v2npl; mkdir -p $O
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -q -k "v2" --timeout 300 --timeout-method thread > $O/pytest_v2.log 2>&1 || { tail -40 $O/pytest_v2.log; exit 1; }
tail -n 2 $O/pytest_v2.log
for v in ${VARS:-v2batch v2nobatch}; do
  FOGNET_LIB=build/live/$v/libfognet_hip.so timeout -k 10 300 python tools/v2_nodes_timing.py 64 ${STOP:-5} ${NS:-65 300 1024} > $O/t_$v.log 2>&1 || { tail $O/t_$v.log; exit 1; }
  echo "== $v"; cat $O/t_$v.log
done
