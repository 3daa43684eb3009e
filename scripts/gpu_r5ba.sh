# Philox pixels per group for full frames with three in flight: 4 (default) vs 8 vs 2 (C5, C4).
set -o pipefail
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 20 --timeout 200 --out gpurun_out/r5ba_ab.jsonl \
  --env wp4="" --env wp8="NRT_WAVE_PIXELS=8" --env wp2="NRT_WAVE_PIXELS=2" \
  --cfg c5="" --cfg c4="--scene scenes/utah-teapot-scene.json"
