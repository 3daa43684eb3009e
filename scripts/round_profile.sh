# Round profile: kernel-trace/stats + PMC passes for the headline kernel and every
# single-GPU BASELINE config's default kernel, plus the reference-exact kernel.
# usage: bash scripts/round_profile.sh <round-tag>   (then: python scripts/publish_profiles.py <round-tag> --as <round-tag>)
set -o pipefail
tag=${1:-r02}
bash scripts/profile.sh ${tag}_c5_f32_philox --steps 3 --warmup 1 && \
bash scripts/profile.sh ${tag}_c4_f32_philox --scene scenes/utah-teapot-scene.json --steps 3 --warmup 1 && \
bash scripts/profile.sh ${tag}_c3_f32_philox --scene scenes/earth.toml --width 1920 --height 1080 --spp 128 --steps 3 --warmup 1 && \
bash scripts/profile.sh ${tag}_c2_f32_philox --width 512 --height 512 --spp 64 --steps 3 --warmup 1 && \
bash scripts/profile.sh ${tag}_c5_f64_chacha8 --precision f64 --rng chacha8 --steps 2 --warmup 1 && \
bash scripts/profile.sh ${tag}_c4_f64_chacha8 --scene scenes/utah-teapot-scene.json --spp 16 --precision f64 --rng chacha8 --steps 2 --warmup 1
