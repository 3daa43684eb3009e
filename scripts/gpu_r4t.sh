# Scheduler strategies: JIT kernels via NRT_JIT_LLVM (C5, C3, C2 world list; C4 world BVH), and the
# hipcc-built generic / exact kernels via experiment libraries (f64 C5 / C4 / C3, C1 1080p generic).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 800 python scripts/ab_configs.py --reps 2 --steps 3 --out gpurun_out/r4t_ab1.jsonl \
  --env base="" --env imo="NRT_JIT_LLVM=-amdgpu-sched-strategy=iterative-maxocc" \
  --cfg c5="" --cfg c3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 128" \
  --cfg c2="--scene scenes/cornell-box-scene.json --width 512 --height 512 --spp 64" || exit 1
timeout -k 10 500 python scripts/ab_configs.py --reps 2 --steps 3 --out gpurun_out/r4t_ab2.jsonl \
  --env ilp="" --env iilp="NRT_JIT_LLVM=-amdgpu-sched-strategy=iterative-ilp" --env imo="NRT_JIT_LLVM=-amdgpu-sched-strategy=iterative-maxocc" \
  --cfg c4="--scene scenes/utah-teapot-scene.json" || exit 1
timeout -k 10 1000 python scripts/ab_configs.py --reps 1 --steps 2 --out gpurun_out/r4t_ab3.jsonl \
  --lib cur=nr-ray-tracer_amd/nrt/libnrt.so --lib xilp=nr-ray-tracer_amd/ab/xilp/libnrt.so --lib xmo=nr-ray-tracer_amd/ab/xmo/libnrt.so \
  --cfg c5f64="--precision f64 --rng chacha8 --steps 1" --cfg c4f64="--scene scenes/utah-teapot-scene.json --precision f64 --rng chacha8 --steps 1" \
  --cfg c3f64="--scene scenes/earth.toml --width 1920 --height 1080 --spp 16 --precision f64 --rng chacha8" \
  --cfg c1big="--scene scenes/spheres.toml --width 1920 --height 1080 --spp 64" || exit 1
echo r4t done
