# Teapot sample pool at 8 pixels per group: ring slots 4 (default) vs 3 / 2 (library builds), and 2
# groups per queue atomic (scene-specialised kernel, NRT_JIT_DEFS).
set -o pipefail
L=nr-ray-tracer_amd
timeout -k 10 900 python scripts/ab_configs.py --reps 3 --steps 12 --timeout 200 --out gpurun_out/r5bd_ab.jsonl \
  --arm s4=$L/nrt/libnrt.so --arm s3=$L/ab/s3/libnrt.so --arm s2=$L/ab/s2/libnrt.so --arm g2="$L/nrt/libnrt.so::NRT_JIT_DEFS=-DNRT_GRAB=2" \
  --cfg c4="--scene scenes/utah-teapot-scene.json"
