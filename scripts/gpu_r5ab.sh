# Exact kernel: phase profile of the persistent walk (C5), candidate-list size 2 / 3 vs 4, and 2 waves
# per SIMD for the LDS-stack variants (alternating A/B on C5 / C4 f64).
set -o pipefail
tag=${1:-r5ab}
mkdir -p gpurun_out
L=nr-ray-tracer_amd
NRT_LIB=$PWD/$L/ab/prof/libnrt.so timeout -k 10 120 python scripts/phase_profile.py scenes/cornell-box-scene.json f64/chacha8/auto > gpurun_out/${tag}_phase_c5.json || exit 1
cat gpurun_out/${tag}_phase_c5.json
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 4 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --arm cur=$L/nrt/libnrt.so --arm xc2=$L/ab/xc2/libnrt.so --arm xc3=$L/ab/xc3/libnrt.so --arm w2=$L/ab/w2/libnrt.so \
  --cfg c5f64="--precision f64 --rng chacha8" --cfg c4f64="--precision f64 --rng chacha8 --scene scenes/utah-teapot-scene.json"
