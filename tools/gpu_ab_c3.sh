set -o pipefail
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/ab
for v in base actmask base actmask; do
  FOGNET_LIB=build/var/$v/libfognet_hip.so FOGNET_STAGES=replay,all timeout -k 10 120 python tools/stage_timing.py 2>&1 | grep -v amdgpu.ids || exit 1
done
