# Bench every BASELINE config that runs on one GPU (C2, C3, C4, C5) plus C1's scene at a GPU size.
# usage: bash scripts/configs_bench.sh <tag>
set -o pipefail
tag=${1:-cfg}
mkdir -p gpurun_out
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/${tag}_$name.json 2> gpurun_out/${tag}_$name.err || { echo "bench $name failed rc=$?"; tail -3 gpurun_out/${tag}_$name.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Msamples/s', d['roofline']['kernel_ms'], 'ms', d['config'].get('trace'), d['config'].get('world_prims'))" gpurun_out/${tag}_$name.json $name
}
run c2_f32 --scene scenes/cornell-box-scene.json --width 512 --height 512 --spp 64 && \
run c3_f32 --scene scenes/earth.toml --width 1920 --height 1080 --spp 128 && \
run c3_f64 --scene scenes/earth.toml --width 1920 --height 1080 --spp 8 --precision f64 --rng chacha8 && \
run c4_f32 --scene scenes/utah-teapot-scene.json && \
run c4_f32_chacha --scene scenes/utah-teapot-scene.json --rng chacha8 --steps 8 && \
run c4_f64 --scene scenes/utah-teapot-scene.json --precision f64 --rng chacha8 --steps 4 && \
run c1_f32 --scene scenes/spheres.toml --width 400 --height 225 --spp 16 && \
run c1_f32_big --scene scenes/spheres.toml --width 1920 --height 1080 --spp 64 && \
run c1_f64 --scene scenes/spheres.toml --width 400 --height 225 --spp 16 --precision f64 --rng chacha8 --steps 8 && \
run c1_f64_big --scene scenes/spheres.toml --width 1920 --height 1080 --spp 64 --precision f64 --rng chacha8 --steps 4 && \
run c5_f32 && \
run c5_f32_chacha --rng chacha8 --steps 8 && \
run c5_f64_chacha --precision f64 --rng chacha8 --steps 4 && \
run c5_f32_bvh --trace bvh && \
{ timeout -k 10 200 python bench.py --cpu-only --scene scenes/spheres.toml --width 400 --height 225 --spp 16 --cpu-row-stride 1 > gpurun_out/${tag}_c1_cpu.json 2> gpurun_out/${tag}_c1_cpu.err && \
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('c1_cpu', d['value'], 'Msamples/s on', d['cpu_baseline']['cores'], 'cores')" gpurun_out/${tag}_c1_cpu.json; }
