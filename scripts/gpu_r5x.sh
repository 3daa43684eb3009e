# Exact kernel: the prefiltered walk kept across shading rounds (XWalk, default) vs one walk per
# segment (NRT_EXACT_PERSIST=0), and the shading-round threshold; exact parity tests first.
set -o pipefail
tag=${1:-r5x}
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden_images.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest.log
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 4 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --env p32="" --env p16="NRT_WAVE_WAIT=16" --env p48="NRT_WAVE_WAIT=48" --env off="NRT_EXACT_PERSIST=0" \
  --cfg c5f64="--precision f64 --rng chacha8" --cfg c4f64="--precision f64 --rng chacha8 --scene scenes/utah-teapot-scene.json"
