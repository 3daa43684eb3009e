# Two groups per queue atomic (NRT_GRAB=2, scene-specialised kernels) vs one: C5, C4, C3, 4 alternating runs.
set -o pipefail
timeout -k 10 1000 python scripts/ab_configs.py --reps 4 --steps 20 --timeout 200 --out gpurun_out/r5bh_ab.jsonl \
  --env g1="" --env g2="NRT_JIT_DEFS=-DNRT_GRAB=2" \
  --cfg c5="" --cfg c4="--scene scenes/utah-teapot-scene.json" --cfg c3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 128"
