# Exact (f64 / ChaCha8) kernel experiments: the phase profile of the LDS-stack planes variant, and
# alternating A/B of paired rejection rounds, FMA contraction in the culling walk, and a stand-in
# for the ChaCha8 block (attribution only: frames differ) on C5 / C4 f64.
set -o pipefail
tag=${1:-r5s}
mkdir -p gpurun_out
NRT_LIB=$PWD/nr-ray-tracer_amd/ab/prof/libnrt.so timeout -k 10 120 python scripts/phase_profile.py scenes/cornell-box-scene.json f64/chacha8/auto > gpurun_out/${tag}_phase_c5.json || exit 1
cat gpurun_out/${tag}_phase_c5.json
L=nr-ray-tracer_amd
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 4 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --arm base=$L/nrt/libnrt.so --arm pair=$L/ab/pair/libnrt.so --arm fma=$L/ab/fma/libnrt.so --arm fake=$L/ab/fake/libnrt.so \
  --cfg c5f64="--precision f64 --rng chacha8" --cfg c4f64="--precision f64 --rng chacha8 --scene scenes/utah-teapot-scene.json"
