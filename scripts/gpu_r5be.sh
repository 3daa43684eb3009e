# Refresh the C4 f32 profile (8 Philox pixels per group).
set -o pipefail
rm -rf gpurun_out/prof_r05_c4_f32_philox
bash scripts/profile.sh r05_c4_f32_philox --scene scenes/utah-teapot-scene.json --steps 12 --warmup 3 || exit 1
python3 scripts/trace_period.py gpurun_out/prof_r05_c4_f32_philox/trace --json gpurun_out/prof_r05_c4_f32_philox/trace_period.json
