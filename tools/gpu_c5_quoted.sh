#!/bin/bash
# C5 bench lines that quote the committed kernel-trace sidecars (profiles/kernel_profile_c5*.json of
# this library), then the PMC passes (tools/gpu_final.sh PART=2); outputs under gpurun_out/final/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/final; mkdir -p $O
timeout -k 10 200 python bench.py --workload c5 > $O/b_c5.log 2>&1 || exit 1
timeout -k 10 200 python bench.py --workload c5 --policy REF_V3 > $O/b_c5_REF_V3.log 2>&1 || exit 1
timeout -k 10 300 python bench.py --workload c5 --c5-recipe saturate --steps 3 --warmup 1 --no-cpu > $O/b_c5_saturate.log 2>&1 || exit 1
[ "${PMC:-1}" = 1 ] && { PART=2 timeout -k 10 800 bash tools/gpu_final.sh > gpurun_out/final2.log 2>&1 || exit 1; }
echo done
