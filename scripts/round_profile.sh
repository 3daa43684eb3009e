# Round profile: kernel-trace/stats + PMC passes (scripts/profile.sh) for every single-GPU
# BASELINE config's default kernel and the reference-exact kernel, in parts that each fit one
# gpurun call.  usage: bash scripts/round_profile.sh <round-tag> f32a|f32b|f64
#   then: python scripts/publish_profiles.py <round-tag> --as <round-tag>
set -o pipefail
tag=${1:-r04}
part=${2:-f32a}
case "$part" in
f32a)
bash scripts/profile.sh ${tag}_c5_f32_philox --steps 20 --warmup 2 && \
bash scripts/profile.sh ${tag}_c4_f32_philox --scene scenes/utah-teapot-scene.json --steps 8 --warmup 2 && \
bash scripts/profile.sh ${tag}_c3_f32_philox --scene scenes/earth.toml --width 1920 --height 1080 --spp 128 --steps 3 --warmup 1 ;;
f32b)
bash scripts/profile.sh ${tag}_c2_f32_philox --width 512 --height 512 --spp 64 --steps 5 --warmup 1 && \
bash scripts/profile.sh ${tag}_c1_f32_philox --scene scenes/spheres.toml --width 400 --height 225 --spp 16 --steps 5 --warmup 1 && \
bash scripts/profile.sh ${tag}_c1big_f32_philox --scene scenes/spheres.toml --width 1920 --height 1080 --spp 64 --steps 3 --warmup 1 ;;
f64)
bash scripts/profile.sh ${tag}_c5_f64_chacha8 --precision f64 --rng chacha8 --steps 2 --warmup 1 && \
bash scripts/profile.sh ${tag}_c4_f64_chacha8 --scene scenes/utah-teapot-scene.json --precision f64 --rng chacha8 --steps 2 --warmup 1 && \
bash scripts/profile.sh ${tag}_c3_f64_chacha8 --scene scenes/earth.toml --width 1920 --height 1080 --spp 16 --precision f64 --rng chacha8 --steps 2 --warmup 1 ;;
esac
