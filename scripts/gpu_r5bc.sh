# World-BVH kernels at >= 8 pixels per group (current) vs the last commit (C4, C1 big, C4 f32 ChaCha8).
set -o pipefail
L=nr-ray-tracer_amd
timeout -k 10 900 python scripts/ab_configs.py --reps 3 --steps 12 --timeout 200 --out gpurun_out/r5bc_ab.jsonl \
  --arm cur=$L/nrt/libnrt.so --arm prev=$L/ab/prev/libnrt.so \
  --cfg c4="--scene scenes/utah-teapot-scene.json" --cfg c1big="--scene scenes/spheres.toml --width 1920 --height 1080 --spp 64"
