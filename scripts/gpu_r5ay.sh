# Shard scaling (pipelined, 24 launches): 4 streams; 3 streams with 4 / 1 pixels per group.
set -o pipefail
mkdir -p gpurun_out
for cfg in "4 0" "3 4" "3 1"; do
  set -- $cfg
  if [ "$2" = "0" ]; then unset NRT_WAVE_PIXELS; else export NRT_WAVE_PIXELS=$2; fi
  SHARD_K=24 SHARD_STREAMS=$1 timeout -k 10 300 python scripts/shard_timing.py > gpurun_out/r5ay_s$1_wp$2.json || exit 1
  python3 -c "
import json,sys
d=json.load(open(sys.argv[1]))
print(sys.argv[1], {k: (v['efficiency_pipelined'], v['shard_ms_pipelined']) for k, v in d.items() if k.startswith('N=')})" gpurun_out/r5ay_s$1_wp$2.json
done
