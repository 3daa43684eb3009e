# ChaCha8 ring top-up at the persistent loop's head vs the samplers' refills only, and the exact walk
# as if-if trips (NRT_EXACT_IFIF 1 / 2), A/B alternating; f64 parity of the candidate libraries first.
set -o pipefail
tag=${1:-r5j}
mkdir -p gpurun_out
export NRT_JIT_CACHE=$PWD/gpurun_out/${tag}_jitcache
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "f64 or chacha or exact" --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -1 gpurun_out/${tag}_pytest.log
for x in xif1 xif2; do
  NRT_LIB=$PWD/nr-ray-tracer_amd/ab/$x/libnrt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "f64 and not jit" --timeout 200 --timeout-method thread > gpurun_out/${tag}_pytest_$x.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest_$x.log; exit 1; }
  tail -1 gpurun_out/${tag}_pytest_$x.log
done
L=nr-ray-tracer_amd
timeout -k 10 1200 python scripts/ab_configs.py --reps 2 --steps 2 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --arm top=$L/nrt/libnrt.so:: --arm notop="$L/ab/notop/libnrt.so::NRT_JIT_DEFS=-DNRT_CHACHA_TOPUP=0" \
  --arm xif1=$L/ab/xif1/libnrt.so:: --arm xif2=$L/ab/xif2/libnrt.so:: \
  --cfg c5f64="--precision f64 --rng chacha8" --cfg c4f64="--scene scenes/utah-teapot-scene.json --precision f64 --rng chacha8" \
  --cfg c3f64="--scene scenes/earth.toml --width 1920 --height 1080 --spp 16 --precision f64 --rng chacha8" || exit 1
timeout -k 10 600 python scripts/ab_configs.py --reps 2 --steps 3 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --arm top=$L/nrt/libnrt.so:: --arm notop="$L/ab/notop/libnrt.so::NRT_JIT_DEFS=-DNRT_CHACHA_TOPUP=0" \
  --cfg c5f32c="--rng chacha8" --cfg c4f32c="--scene scenes/utah-teapot-scene.json --rng chacha8" || exit 1
