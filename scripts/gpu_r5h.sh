# SGPR-pressure variants of the world-list kernel (scene-specialised, NRT_JIT_DEFS), alternating.
set -o pipefail
tag=${1:-r5h}
mkdir -p gpurun_out
export NRT_JIT_CACHE=$PWD/gpurun_out/${tag}_jitcache
L=nr-ray-tracer_amd/nrt/libnrt.so
timeout -k 10 1000 python scripts/ab_configs.py --reps 3 --steps 10 --out gpurun_out/${tag}_ab.jsonl \
  --arm base=$L:: --arm c7="$L::NRT_JIT_DEFS=-DNRT_CAM_RELOAD=1" \
  --arm r7="$L::NRT_JIT_DEFS=-DNRT_CAM_RELOAD=1 -DNRT_WL_RELOAD=1" \
  --arm c8="$L::NRT_JIT_DEFS=-DNRT_CAM_RELOAD=1 -DNRT_FLAT_WAVES=8" \
  --cfg c5="" --cfg c3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 128" || exit 1
