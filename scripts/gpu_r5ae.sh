# ChaCha8 with the stream's zero high word folded (current) vs the previous commit; stream parity.
set -o pipefail
tag=${1:-r5ae}
mkdir -p gpurun_out
L=nr-ray-tracer_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden_images.py tests/test_library.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -1 gpurun_out/${tag}_pytest.log
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 4 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --arm cur=$L/nrt/libnrt.so --arm prev=$L/ab/prev/libnrt.so \
  --cfg c5f64="--precision f64 --rng chacha8" --cfg c4f64="--precision f64 --rng chacha8 --scene scenes/utah-teapot-scene.json" \
  --cfg c3f64="--precision f64 --rng chacha8 --scene scenes/earth.toml --width 1920 --height 1080 --spp 8" --cfg c5f32c="--rng chacha8"
