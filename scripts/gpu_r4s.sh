# max-ILP scheduling for the world-BVH scene-specialised kernels: suite, alternating timing vs the
# previous build (C4 Philox, C4 f32 ChaCha8, C5 unchanged), full-frame JIT/generic comparison.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4s_pytest.log 2>&1 || { tail -30 gpurun_out/r4s_pytest.log; exit 1; }
tail -2 gpurun_out/r4s_pytest.log
timeout -k 10 200 python scripts/jit_compare.py > gpurun_out/r4s_jit_compare.log 2>&1; rc=$?; tail -8 gpurun_out/r4s_jit_compare.log; [ $rc -le 1 ] || exit 1
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 3 --out gpurun_out/r4s_ab.jsonl \
  --lib new=nr-ray-tracer_amd/nrt/libnrt.so --lib base=nr-ray-tracer_amd/ab/base/libnrt.so \
  --cfg c4="--scene scenes/utah-teapot-scene.json" --cfg c4cc="--scene scenes/utah-teapot-scene.json --rng chacha8 --steps 1" || exit 1
echo r4s done
