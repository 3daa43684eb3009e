# 64-thread workgroups vs 256 (pipelined default bench), C5 and C4.
set -o pipefail
tag=${1:-r5d}
mkdir -p gpurun_out
export NRT_JIT_CACHE=$PWD/gpurun_out/${tag}_jitcache
timeout -k 10 900 python scripts/ab_configs.py --reps 3 --steps 10 --out gpurun_out/${tag}_ab.jsonl \
  --arm b256=nr-ray-tracer_amd/nrt/libnrt.so:: --arm b64="nr-ray-tracer_amd/ab/b64/libnrt.so::NRT_JIT_DEFS=-DNRT_BLOCK=64" \
  --cfg c5="" --cfg c4="--scene scenes/utah-teapot-scene.json" --cfg c3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 128" || exit 1
