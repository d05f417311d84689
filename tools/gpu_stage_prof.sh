set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out
FOGNET_STAGES=all,replay,all,replay timeout -k 10 200 python tools/stage_timing.py > gpurun_out/stage.log 2>&1 || exit 1
timeout -k 10 200 python tools/replay_counters.py --mode time --R 4096 --ring 2048 --out gpurun_out/cyc.json > /dev/null 2>gpurun_out/cyc.err || exit 1
timeout -k 10 200 python tools/replay_counters.py --R 4096 --ring 2048 --out gpurun_out/cnt.json > /dev/null 2>gpurun_out/cnt.err || exit 1
cat gpurun_out/stage.log; python3 -c "import json; d=json.load(open('gpurun_out/cyc.json'))['all']; print({k: round(v,1) for k,v in d.items()})"
