# C4 f64: current library vs commit 9121f89 (ChaCha8 fold) on one box (regression check).
set -o pipefail
L=nr-ray-tracer_amd
timeout -k 10 900 python scripts/ab_configs.py --reps 3 --steps 4 --timeout 200 --out gpurun_out/r5bj_ab.jsonl \
  --arm cur=$L/nrt/libnrt.so --arm old=$L/ab/prev/libnrt.so \
  --cfg c4f64="--precision f64 --rng chacha8 --scene scenes/utah-teapot-scene.json"
