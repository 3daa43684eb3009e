# Persistent exact walk: shading-round threshold 48 / 56 / 60 / 64 vs one walk per segment.
set -o pipefail
tag=${1:-r5y}
mkdir -p gpurun_out
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 4 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --env p48="NRT_WAVE_WAIT=48" --env p56="NRT_WAVE_WAIT=56" --env p60="NRT_WAVE_WAIT=60" --env p64="NRT_WAVE_WAIT=64" --env off="NRT_EXACT_PERSIST=0" \
  --cfg c4f64="--precision f64 --rng chacha8 --scene scenes/utah-teapot-scene.json" --cfg c5f64="--precision f64 --rng chacha8"
