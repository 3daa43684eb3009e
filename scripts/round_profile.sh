# Round profile: kernel-trace/stats + PMC passes for the headline kernel (f32 philox)
# and the reference-exact kernel (f64 chacha8), then the default bench line (with cpu_baseline).
# usage: bash scripts/round_profile.sh <round-tag>
set -o pipefail
tag=${1:-r01}
bash scripts/profile.sh ${tag}_f32_philox --steps 3 --warmup 1 --precision f32 --rng philox && \
bash scripts/profile.sh ${tag}_f64_chacha8 --steps 2 --warmup 1 --precision f64 --rng chacha8 && \
timeout -k 10 400 python bench.py > gpurun_out/${tag}_bench_default.json 2> gpurun_out/${tag}_bench_default.err && \
cat gpurun_out/${tag}_bench_default.json
