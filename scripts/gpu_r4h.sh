set -o pipefail
mkdir -p gpurun_out
timeout -k 10 700 python scripts/ab_configs.py --reps 2 --out gpurun_out/r4h_ab_c4.jsonl --lib B=nr-ray-tracer_amd/nrt/libnrt.so \
  --env base="NRT_JIT_DEFS=" --env pf6="NRT_JIT_DEFS=-DNRT_NODE_PREFETCH=1" --env pf5="NRT_JIT_DEFS=-DNRT_NODE_PREFETCH=1 -DNRT_WBVH_WAVES=5" \
  --cfg c4="--scene scenes/utah-teapot-scene.json" 2>&1 | tail -4 || exit 1
timeout -k 10 400 python scripts/ab_configs.py --reps 2 --out gpurun_out/r4h_ab_c5.jsonl --lib B=nr-ray-tracer_amd/nrt/libnrt.so \
  --env w6="NRT_JIT_DEFS=" --env w8="NRT_JIT_DEFS=-DNRT_WORLD_LIST_WAVES=8" --env w7="NRT_JIT_DEFS=-DNRT_WORLD_LIST_WAVES=7" \
  --cfg c5="" 2>&1 | tail -4 || exit 1
