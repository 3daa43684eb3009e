# Persistent exact walk with its final defaults vs one walk per segment (C5 / C4 / C2 f64), then the
# exact parity tests.
set -o pipefail
tag=${1:-r5aa}
mkdir -p gpurun_out
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 4 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --env dflt="" --env off="NRT_EXACT_PERSIST=0" \
  --cfg c5f64="--precision f64 --rng chacha8" --cfg c4f64="--precision f64 --rng chacha8 --scene scenes/utah-teapot-scene.json" \
  --cfg c2f64="--precision f64 --rng chacha8 --width 512 --height 512 --spp 64" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden_images.py tests/test_multigpu.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest.log
