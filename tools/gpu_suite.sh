#!/bin/bash
# GPU suite + one bench line (one gpurun call): tools/gpu_suite.sh TAG [bench.py args...]
# The bench runs only after a pytest that finished (rc 0 or 1: tests failed);
# a timeout, abort or fault ends the call there.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=$1; shift
cat /sys/fs/cgroup/cpu.max > gpurun_out/${TAG}_cpu_max.txt 2>/dev/null
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread \
  > gpurun_out/${TAG}_pytest.log 2>&1
rc=$?
echo "pytest rc=$rc" >> gpurun_out/${TAG}_pytest.log
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 300 python bench.py "$@" > gpurun_out/${TAG}_bench.json 2> gpurun_out/${TAG}_bench.err
