# Warm-up count vs the wall time per step (stream queues created before the timed region).
set -o pipefail
tag=${1:-r5r}
mkdir -p gpurun_out
for r in 1 2; do
  for w in 2 5; do
    for cfg in "c5|" "c2|--width 512 --height 512 --spp 64"; do
      name=${cfg%%|*}; args=${cfg#*|}
      timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup $w $args > gpurun_out/${tag}_${name}_w${w}_$r.json 2>/dev/null || exit 1
      python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read())
print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" gpurun_out/${tag}_${name}_w${w}_$r.json ${name}_w$w
    done
  done
done
