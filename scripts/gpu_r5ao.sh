# Spheres scene through the exact kernel: the compact walk with its stack in LDS (new EXACT_SIG_WORLD
# variant) vs the last commit's generic kernel (scratch stack); exact parity first.
set -o pipefail
tag=${1:-r5ao}
mkdir -p gpurun_out
L=nr-ray-tracer_amd
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden_images.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -1 gpurun_out/${tag}_pytest.log
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 4 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --arm cur=$L/nrt/libnrt.so --arm prev=$L/ab/prev/libnrt.so \
  --cfg c1bigf64="--precision f64 --rng chacha8 --scene scenes/spheres.toml --width 1920 --height 1080 --spp 64" \
  --cfg c1f64="--precision f64 --rng chacha8 --scene scenes/spheres.toml --width 400 --height 225 --spp 16"
