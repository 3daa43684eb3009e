# Exact kernel: wave-converged rejection samplers (NRT_RIUS_WAVE) with / without the loop-head
# top-up, and FMA contraction in the culling walk alone, against the default library (alternating).
set -o pipefail
tag=${1:-r5t}
mkdir -p gpurun_out
L=nr-ray-tracer_amd
timeout -k 10 1000 python scripts/ab_configs.py --reps 2 --steps 4 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --arm base=$L/nrt/libnrt.so --arm fma=$L/ab/fma/libnrt.so --arm wave=$L/ab/wave/libnrt.so --arm wavent=$L/ab/wavent/libnrt.so \
  --cfg c5f64="--precision f64 --rng chacha8" --cfg c4f64="--precision f64 --rng chacha8 --scene scenes/utah-teapot-scene.json" \
  --cfg c3f64="--precision f64 --rng chacha8 --scene scenes/earth.toml --width 1920 --height 1080 --spp 8" \
  --cfg c5f32c="--rng chacha8"
