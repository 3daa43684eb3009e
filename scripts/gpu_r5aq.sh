# Spheres scene, persistent unfiltered exact walk: threshold 56 (default) / 60 / 64 / 48.
set -o pipefail
tag=${1:-r5aq}
mkdir -p gpurun_out
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 4 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --env p56="" --env p48="NRT_WAVE_WAIT=48" --env p60="NRT_WAVE_WAIT=60" --env p64="NRT_WAVE_WAIT=64" \
  --cfg c1bigf64="--precision f64 --rng chacha8 --scene scenes/spheres.toml --width 1920 --height 1080 --spp 64"
