# Exact C5 f64: phase profile with the walk / candidate-test split and walk lane events (NRT_EXACT_PROF
# build), and the every-slot prefilter vs the walk now that both use FMAs (alternating).
set -o pipefail
tag=${1:-r5v}
mkdir -p gpurun_out
NRT_LIB=$PWD/nr-ray-tracer_amd/ab/prof/libnrt.so timeout -k 10 120 python scripts/phase_profile.py scenes/cornell-box-scene.json f64/chacha8/auto > gpurun_out/${tag}_phase_c5.json || exit 1
cat gpurun_out/${tag}_phase_c5.json
NRT_LIB=$PWD/nr-ray-tracer_amd/ab/prof/libnrt.so timeout -k 10 120 python scripts/phase_profile.py scenes/utah-teapot-scene.json f64/chacha8/auto > gpurun_out/${tag}_phase_c4.json || exit 1
cat gpurun_out/${tag}_phase_c4.json
timeout -k 10 600 python scripts/ab_configs.py --reps 2 --steps 4 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --env walk="" --env slots="NRT_EXACT_SLOTS=1" --cfg c5f64="--precision f64 --rng chacha8"
