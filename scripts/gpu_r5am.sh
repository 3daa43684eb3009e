# Teapot world BVH build: SAH primitive weight 0.7 / 1 (default) / 1.5 / 2 and leaf bound 2 / 3 vs 4
# (host build knobs), f32 and f64 (alternating).
set -o pipefail
tag=${1:-r5am}
mkdir -p gpurun_out
timeout -k 10 1000 python scripts/ab_configs.py --reps 2 --steps 8 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --env p1="" --env p07="NRT_SAH_PRIM_COST=0.7" --env p15="NRT_SAH_PRIM_COST=1.5" --env p2="NRT_SAH_PRIM_COST=2" \
  --env l3="NRT_WBVH_LEAF=3" --env l2="NRT_WBVH_LEAF=2" \
  --cfg c4="--scene scenes/utah-teapot-scene.json" || exit 1
timeout -k 10 600 python scripts/ab_configs.py --reps 1 --steps 3 --timeout 200 --out gpurun_out/${tag}_ab64.jsonl \
  --env p1="" --env p15="NRT_SAH_PRIM_COST=1.5" --env p07="NRT_SAH_PRIM_COST=0.7" \
  --cfg c4f64="--precision f64 --rng chacha8 --scene scenes/utah-teapot-scene.json"
