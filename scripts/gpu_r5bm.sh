# Exact kernel pixel claims per counter atomic at spp 256: 1 (default) vs 2 / 4 (C5 / C4 f64).
set -o pipefail
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 4 --timeout 200 --out gpurun_out/r5bm_ab.jsonl \
  --env c1="" --env c2="NRT_EXACT_CLAIM=2" --env c4="NRT_EXACT_CLAIM=4" \
  --cfg c5f64="--precision f64 --rng chacha8" --cfg c4f64="--precision f64 --rng chacha8 --scene scenes/utah-teapot-scene.json"
