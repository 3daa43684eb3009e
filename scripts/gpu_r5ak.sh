# Persistent exact loop: a ChaCha8 top-up at each shading round's head (NRT_XWALK_TOPUP) vs none.
set -o pipefail
tag=${1:-r5ak}
mkdir -p gpurun_out
L=nr-ray-tracer_amd
timeout -k 10 900 python scripts/ab_configs.py --reps 3 --steps 4 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --arm cur=$L/nrt/libnrt.so --arm topup=$L/ab/topup/libnrt.so \
  --cfg c5f64="--precision f64 --rng chacha8" --cfg c4f64="--precision f64 --rng chacha8 --scene scenes/utah-teapot-scene.json"
