# f32 world BVH shading threshold: spheres 48 / 56 / 64, teapot 24 / 32 / 40.
set -o pipefail
tag=${1:-r5aw}
mkdir -p gpurun_out
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 8 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --env w48="NRT_WAVE_WAIT=48" --env w56="NRT_WAVE_WAIT=56" --env w64="NRT_WAVE_WAIT=64" \
  --cfg c1big="--scene scenes/spheres.toml --width 1920 --height 1080 --spp 64" || exit 1
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 12 --timeout 200 --out gpurun_out/${tag}_ab2.jsonl \
  --env w24="" --env w32="NRT_WAVE_WAIT=32" --env w40="NRT_WAVE_WAIT=40" \
  --cfg c4="--scene scenes/utah-teapot-scene.json"
