# Leaf batching in the if-if trips (NRT_LEAF_BATCH, scene-specialised kernels) on C4 / C1-1080p,
# and the host-picked pixel claim of the persistent lanes (f64 C3 / C4).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4k_pytest.log 2>&1 || { tail -30 gpurun_out/r4k_pytest.log; exit 1; }
tail -2 gpurun_out/r4k_pytest.log
timeout -k 10 700 python scripts/ab_configs.py --reps 2 --steps 3 --out gpurun_out/r4k_ab.jsonl \
  --env lb0="" --env lb12="NRT_JIT_DEFS=-DNRT_LEAF_BATCH=12" --env lb24="NRT_JIT_DEFS=-DNRT_LEAF_BATCH=24" --env lb40="NRT_JIT_DEFS=-DNRT_LEAF_BATCH=40" \
  --cfg c4="--scene scenes/utah-teapot-scene.json" || exit 1
timeout -k 10 400 python scripts/ab_configs.py --reps 1 --steps 2 --out gpurun_out/r4k_ab64.jsonl \
  --cfg c3f64="--scene scenes/earth.toml --width 1920 --height 1080 --spp 16 --precision f64 --rng chacha8" \
  --cfg c4f64="--scene scenes/utah-teapot-scene.json --precision f64 --rng chacha8" || exit 1
echo r4k done
