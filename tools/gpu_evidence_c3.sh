#!/bin/bash
# C3 evidence on the current tree: rocprof kernel statistics of the bench, then
# the PMC passes (tools/gpu_pmc.sh).  Outputs under gpurun_out/ev/ and gpurun_out/pmc/.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/ev; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o c3 -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/prof_c3.log 2>&1 || { tail $O/prof_c3.log; exit 1; }
find $O/prof_c3 -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $O/kernel_stats_c3.csv
head -5 $O/kernel_stats_c3.csv
bash tools/gpu_pmc.sh > $O/pmc_c3.log 2>&1 || { tail $O/pmc_c3.log; exit 1; }
tail -3 $O/pmc_c3.log
