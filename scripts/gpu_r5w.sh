# Exact kernel: the small culling tree staged in LDS (default) vs read from global memory
# (NRT_EXACT_XSTAGE=0), alternating; then the exact parity tests.
set -o pipefail
tag=${1:-r5w}
mkdir -p gpurun_out
timeout -k 10 600 python scripts/ab_configs.py --reps 2 --steps 4 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --env xstage="" --env global="NRT_EXACT_XSTAGE=0" --cfg c5f64="--precision f64 --rng chacha8" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_golden_images.py -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest.log
