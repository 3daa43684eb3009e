# Philox group size rule: halve P below 16 (default) vs 4 groups per resident wave: shard scaling
# (pipelined, 8 / 24 launches, 2 / 3 streams) and the C2 / C5 / C4 bench lines.
set -o pipefail
mkdir -p gpurun_out
for g in 16 4; do
  for cfg in "8 2" "24 3"; do
    set -- $cfg
    NRT_GROUPS_PER_WAVE=$g SHARD_K=$1 SHARD_STREAMS=$2 timeout -k 10 300 python scripts/shard_timing.py > gpurun_out/r5az_g${g}_k$1_s$2.json || exit 1
    python3 -c "
import json,sys
d=json.load(open(sys.argv[1]))
print(sys.argv[1], {k: (v['efficiency_pipelined'], v['shard_ms_pipelined']) for k, v in d.items() if k.startswith('N=')})" gpurun_out/r5az_g${g}_k$1_s$2.json
  done
done
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 20 --timeout 200 --out gpurun_out/r5az_ab.jsonl \
  --env g16="" --env g4="NRT_GROUPS_PER_WAVE=4" \
  --cfg c2="--width 512 --height 512 --spp 64" --cfg c5="" --cfg c4="--scene scenes/utah-teapot-scene.json"
