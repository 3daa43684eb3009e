# 4-wide node steps with two mantissa bits vs powers of two: GPU suite, then A/B (alternating).
set -o pipefail
tag=${1:-r5m}
mkdir -p gpurun_out
export NRT_JIT_CACHE=$PWD/gpurun_out/${tag}_jitcache
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -1 gpurun_out/${tag}_pytest.log
L=nr-ray-tracer_amd
timeout -k 10 1200 python scripts/ab_configs.py --reps 3 --steps 12 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --arm base=$L/ab/base/libnrt.so:: --arm mant=$L/nrt/libnrt.so:: \
  --cfg c4="--scene scenes/utah-teapot-scene.json" --cfg c1big="--scene scenes/spheres.toml --width 1920 --height 1080 --spp 64" || exit 1
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 3 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --arm base=$L/ab/base/libnrt.so:: --arm mant=$L/nrt/libnrt.so:: \
  --cfg c4f64="--scene scenes/utah-teapot-scene.json --precision f64 --rng chacha8" --cfg c5f64="--precision f64 --rng chacha8" || exit 1
