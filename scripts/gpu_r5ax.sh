# Shard scaling (pipelined) with 8 vs 24 launches per measurement (steady state), 2 and 3 streams.
set -o pipefail
mkdir -p gpurun_out
cd /root/repo
for cfg in "8 2" "24 2" "24 3"; do
  set -- $cfg
  SHARD_K=$1 SHARD_STREAMS=$2 timeout -k 10 300 python scripts/shard_timing.py > gpurun_out/r5ax_k$1_s$2.json || exit 1
  python3 -c "
import json,sys
d=json.load(open(sys.argv[1]))
print(sys.argv[1], {k: v['efficiency_pipelined'] for k, v in d.items() if k.startswith('N=')})" gpurun_out/r5ax_k$1_s$2.json
done
