# Profile of the spheres scene through the exact kernel (persistent unfiltered walk).
set -o pipefail
rm -rf gpurun_out/prof_r05_c1big_f64_chacha8
bash scripts/profile.sh r05_c1big_f64_chacha8 --scene scenes/spheres.toml --width 1920 --height 1080 --spp 64 --precision f64 --rng chacha8 --steps 3 --warmup 1 || exit 1
python3 scripts/trace_period.py gpurun_out/prof_r05_c1big_f64_chacha8/trace --json gpurun_out/prof_r05_c1big_f64_chacha8/trace_period.json > /dev/null || true
