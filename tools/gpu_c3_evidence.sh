#!/bin/bash
# C3 evidence on the current tree: bench line (20 steps), rocprof kernel stats, PMC passes + calibration.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/c3ev; mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python bench.py --gpus 1 --steps 20 --warmup 5 > $O/bench_c3.log 2>&1 || { tail $O/bench_c3.log; exit 1; }
grep '^{' $O/bench_c3.log | tail -n 1 > $O/bench_c3.json
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3 -o c3 -- python3 bench.py --steps 5 --warmup 1 --no-cpu > $O/prof_c3.log 2>&1 || { tail $O/prof_c3.log; exit 1; }
bash tools/gpu_pmc.sh > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
cp gpurun_out/pmc/pmc_traffic.json $O/
echo done
