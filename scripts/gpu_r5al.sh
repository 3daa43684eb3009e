# C4 f32 world-BVH kernel at 6 (default) / 7 / 8 waves per SIMD (scene-specialised, NRT_JIT_DEFS).
set -o pipefail
tag=${1:-r5al}
mkdir -p gpurun_out
timeout -k 10 900 python scripts/ab_configs.py --reps 3 --steps 12 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --env w6="" --env w7="NRT_JIT_DEFS=-DNRT_WBVH_WAVES=7" --env w8="NRT_JIT_DEFS=-DNRT_WBVH_WAVES=8" \
  --cfg c4="--scene scenes/utah-teapot-scene.json"
