set -o pipefail
STAGES=replay,all bash tools/ab.sh base inlq2 > gpurun_out/ab.log 2>&1 || exit 1
VARIANTS="base inlq inlq2" bash tools/gpu_ab_c4.sh
