# Round-4 evidence: earth f64 profile after the pixel claims, every single-GPU config, shard timing,
# the default bench line (with the CPU baseline).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
bash scripts/profile.sh r04_c3_f64_chacha8 --scene scenes/earth.toml --width 1920 --height 1080 --spp 16 --precision f64 --rng chacha8 --steps 2 --warmup 1 || exit 1
bash scripts/configs_bench.sh r04_cfg || exit 1
timeout -k 10 200 python scripts/shard_timing.py > gpurun_out/r04_shard_c5.json 2> gpurun_out/r04_shard_c5.err || exit 1
timeout -k 10 300 python bench.py > gpurun_out/r04_bench_default.json 2> gpurun_out/r04_bench_default.err || exit 1
echo r4l done
