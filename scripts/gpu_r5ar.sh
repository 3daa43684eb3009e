# Exact prefilter with one live candidate (NRT_XCAND=1) vs two.
set -o pipefail
tag=${1:-r5ar}
mkdir -p gpurun_out
L=nr-ray-tracer_amd
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 4 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --arm x2=$L/nrt/libnrt.so --arm x1=$L/ab/xc1/libnrt.so \
  --cfg c5f64="--precision f64 --rng chacha8" --cfg c4f64="--precision f64 --rng chacha8 --scene scenes/utah-teapot-scene.json"
