# Persistent exact loop: camera rays with the disk drawn at the converged loop head (current) vs the
# last commit (alternating, 3 reps).
set -o pipefail
tag=${1:-r5ah}
mkdir -p gpurun_out
L=nr-ray-tracer_amd
timeout -k 10 900 python scripts/ab_configs.py --reps 3 --steps 4 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --arm cur=$L/nrt/libnrt.so --arm prev=$L/ab/prev/libnrt.so \
  --cfg c5f64="--precision f64 --rng chacha8" --cfg c4f64="--precision f64 --rng chacha8 --scene scenes/utah-teapot-scene.json"
