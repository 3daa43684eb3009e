# Spheres scene, f32 world BVH: the scene-specialised kernel (NRT_JIT_WBVH_ANY=1) vs the generic one.
set -o pipefail
tag=${1:-r5au}
mkdir -p gpurun_out
timeout -k 10 900 python scripts/ab_configs.py --reps 3 --steps 8 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --env gen="" --env jit="NRT_JIT_WBVH_ANY=1" \
  --cfg c1big="--scene scenes/spheres.toml --width 1920 --height 1080 --spp 64"
