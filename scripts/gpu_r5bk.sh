# Refresh the headline C5 profile with the final library (two groups per queue atomic).
set -o pipefail
rm -rf gpurun_out/prof_r05_c5_f32_philox
bash scripts/profile.sh r05_c5_f32_philox --steps 20 --warmup 2 || exit 1
python3 scripts/trace_period.py gpurun_out/prof_r05_c5_f32_philox/trace --json gpurun_out/prof_r05_c5_f32_philox/trace_period.json
