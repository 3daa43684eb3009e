# Philox pixels per group, full frames: C4 8 / 16 / 32, C5 8 / 16, C2 default vs 16 / 32.
set -o pipefail
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 12 --timeout 200 --out gpurun_out/r5bb_ab.jsonl \
  --env wp8="NRT_WAVE_PIXELS=8" --env wp16="NRT_WAVE_PIXELS=16" --env wp32="NRT_WAVE_PIXELS=32" \
  --cfg c4="--scene scenes/utah-teapot-scene.json" || exit 1
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 20 --timeout 200 --out gpurun_out/r5bb_ab2.jsonl \
  --env dflt="" --env wp16="NRT_WAVE_PIXELS=16" --env wp32="NRT_WAVE_PIXELS=32" \
  --cfg c5="" --cfg c1big="--scene scenes/spheres.toml --width 1920 --height 1080 --spp 64" --cfg c3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 128"
