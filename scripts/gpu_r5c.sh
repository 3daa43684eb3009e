# NRT_NODE_MIX A/B on C4 (alternating, scene-specialised arms only) + one-shot CLI timing.
set -o pipefail
tag=${1:-r5c}
mkdir -p gpurun_out
export NRT_JIT_CACHE=$PWD/gpurun_out/${tag}_jitcache
timeout -k 10 600 python scripts/ab_configs.py --reps 3 --steps 5 --out gpurun_out/${tag}_ab.jsonl \
  --env base="" --env mix="NRT_JIT_DEFS=-DNRT_NODE_MIX=1" \
  --cfg c4="--scene scenes/utah-teapot-scene.json" || exit 1
cd tests/golden
TIMEFORMAT="cli wall %R s"
for run in 1 2; do
  time timeout -k 10 120 ../../nr-ray-tracer_amd/nrt/nrt-cli render scenes/cornell-box-scene.json -W 1024 -H 1024 --samples-per-pixel 256 --precision f32 --rng philox -v -f -o /tmp/c5.png
done
