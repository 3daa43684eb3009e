# Spheres scene: the unfiltered exact walk kept across shading rounds (XWalkU) at thresholds 24 / 40 /
# 56 vs one walk per segment; exact parity first.
set -o pipefail
tag=${1:-r5ap}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden_images.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -1 gpurun_out/${tag}_pytest.log
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 4 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --env p40="" --env p24="NRT_WAVE_WAIT=24" --env p56="NRT_WAVE_WAIT=56" --env off="NRT_EXACT_PERSIST=0" \
  --cfg c1bigf64="--precision f64 --rng chacha8 --scene scenes/spheres.toml --width 1920 --height 1080 --spp 64" \
  --cfg c1f64="--precision f64 --rng chacha8 --scene scenes/spheres.toml --width 400 --height 225 --spp 16"
