# Headline world-list kernel: 2 groups per queue atomic, no head probe (scene-specialised, NRT_JIT_DEFS).
set -o pipefail
timeout -k 10 900 python scripts/ab_configs.py --reps 3 --steps 20 --timeout 200 --out gpurun_out/r5bg_ab.jsonl \
  --env dflt="" --env g2="NRT_JIT_DEFS=-DNRT_GRAB=2" --env np="NRT_JIT_DEFS=-DNRT_PROBE_HEAD=0" \
  --cfg c5=""
