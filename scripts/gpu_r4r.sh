# Scheduler strategies for the scene-specialised kernels (NRT_JIT_LLVM), C5 and C4.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 1000 python scripts/ab_configs.py --reps 2 --steps 3 --out gpurun_out/r4r_ab.jsonl \
  --env base="" --env mclause="NRT_JIT_LLVM=-amdgpu-sched-strategy=max-memory-clause" \
  --env ilp="NRT_JIT_LLVM=-amdgpu-sched-strategy=max-ilp" \
  --env nounc="NRT_JIT_LLVM=-amdgpu-disable-unclustered-high-rp-reschedule" \
  --cfg c5="" --cfg c4="--scene scenes/utah-teapot-scene.json" || exit 1
echo r4r done
