set -o pipefail
mkdir -p gpurun_out/r5
for v in ${VARS:-rbase fnoe fnos}; do
  FOGNET_LIB=build/live/$v/libfognet_hip.so POWER=$POWER WORKLOAD=c5 POLICY=EXT_HIER FOGNET_STAGES=all,all timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/r5/ktf_$v -o k -- python3 tools/stage_timing.py 1024 > gpurun_out/r5/ktf_$v.log 2>&1 || exit 1
  python3 tools/kstats.py gpurun_out/r5/ktf_$v --skip 2 --out gpurun_out/r5/ktf_$v.csv || exit 1
  echo "== $v"; python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/r5/ktf_$v.csv')):
    if 'region' in r['Name']: print('  ', r['Name'][:60], r['Calls'], round(float(r['AverageNs'])/1e3,1), 'us')"
done
