# Spheres scene, f32 world BVH: shading threshold 32 (default) / 40 / 48.
set -o pipefail
tag=${1:-r5av}
mkdir -p gpurun_out
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 8 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --env w32="" --env w40="NRT_WAVE_WAIT=40" --env w48="NRT_WAVE_WAIT=48" \
  --cfg c1big="--scene scenes/spheres.toml --width 1920 --height 1080 --spp 64"
