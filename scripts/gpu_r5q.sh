# Exact kernel every-slot prefilter (NRT_EXACT_SLOTS=1) vs the walk on C5 f64 (alternating), and the C4
# headline-config profile of the final library.
set -o pipefail
tag=${1:-r5q}
mkdir -p gpurun_out
timeout -k 10 900 python scripts/ab_configs.py --reps 2 --steps 4 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --env walk="" --env slots="NRT_EXACT_SLOTS=1" --cfg c5f64="--precision f64 --rng chacha8" || exit 1
rm -rf gpurun_out/prof_r05_c4_f32_philox
bash scripts/profile.sh r05_c4_f32_philox --scene scenes/utah-teapot-scene.json --steps 12 --warmup 3 || exit 1
python3 scripts/trace_period.py gpurun_out/prof_r05_c4_f32_philox/trace --json gpurun_out/prof_r05_c4_f32_philox/trace_period.json
