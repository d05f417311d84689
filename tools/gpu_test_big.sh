set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/big
timeout -k 10 900 python -u -m pytest tests/test_parity_gpu.py -m gpu -x -v -k "wide or unsupported or c5 or down or hier" --timeout 600 --timeout-method thread > gpurun_out/big/pytest.log 2>&1 || { tail -60 gpurun_out/big/pytest.log; exit 1; }
tail -n 3 gpurun_out/big/pytest.log
