# Persistent exact walk: a trip that offers or visits (NRT_XWALK_ONE) vs one that may do both; C4 f32
# shading threshold 20 / 24 / 28 (alternating).
set -o pipefail
tag=${1:-r5aj}
mkdir -p gpurun_out
L=nr-ray-tracer_amd
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 4 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --arm both=$L/nrt/libnrt.so --arm one=$L/ab/one/libnrt.so \
  --cfg c5f64="--precision f64 --rng chacha8" --cfg c4f64="--precision f64 --rng chacha8 --scene scenes/utah-teapot-scene.json" || exit 1
timeout -k 10 900 python scripts/ab_configs.py --reps 3 --steps 12 --timeout 200 --out gpurun_out/${tag}_ab2.jsonl \
  --env w24="" --env w20="NRT_WAVE_WAIT=20" --env w28="NRT_WAVE_WAIT=28" \
  --cfg c4="--scene scenes/utah-teapot-scene.json"
