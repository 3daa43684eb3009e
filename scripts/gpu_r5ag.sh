# f32 world-BVH kernel: compact nodes with f16 planes (NRT_WBVH_HALF, v_fma_mix reads) vs bytes, C4
# (alternating, 3 reps); then the exact-kernel profiles and the configs bench.
set -o pipefail
tag=${1:-r5ag}
mkdir -p gpurun_out
timeout -k 10 900 python scripts/ab_configs.py --reps 3 --steps 12 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --env bytes="" --env half="NRT_JIT_DEFS=-DNRT_WBVH_HALF=1" \
  --cfg c4="--scene scenes/utah-teapot-scene.json" --cfg c1big="--scene scenes/spheres.toml --width 1920 --height 1080 --spp 64" || exit 1
bash scripts/gpu_r5af.sh r5af || exit 1
