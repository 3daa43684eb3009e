# Frames in flight at N = 1: D = 3 (copy stream) vs 4 (copies on the render streams), alternating.
set -o pipefail
tag=${1:-r5p}
mkdir -p gpurun_out
for cfg in "c5|" "c4|--scene scenes/utah-teapot-scene.json" "c2|--width 512 --height 512 --spp 64"; do
  name=${cfg%%|*}; args=${cfg#*|}
  for r in 1 2; do
    for p in 3 4; do
      timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --pipeline $p $args > gpurun_out/${tag}_${name}_p${p}_$r.json 2>/dev/null || exit 1
      python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read())
print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['timings_ms']['d2h_copy'], d['frame_sha256'][:12])" gpurun_out/${tag}_${name}_p${p}_$r.json ${name}_p$p
    done
  done
done
