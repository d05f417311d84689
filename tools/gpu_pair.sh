set -o pipefail
STAGES=replay,all bash tools/ab.sh base pair > gpurun_out/ab_pair.log 2>&1 || exit 1
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pair.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_pair.log
exit $rc
