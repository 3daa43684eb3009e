# World-list sample pool: ring slots 2 (default) vs 3 / 4 (library builds), C5 and C3 with frames in flight.
set -o pipefail
L=nr-ray-tracer_amd
timeout -k 10 900 python scripts/ab_configs.py --reps 3 --steps 20 --timeout 200 --out gpurun_out/r5bf_ab.jsonl \
  --arm l2=$L/nrt/libnrt.so --arm l3=$L/ab/l3/libnrt.so --arm l4=$L/ab/l4/libnrt.so \
  --cfg c5="" --cfg c3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 128"
