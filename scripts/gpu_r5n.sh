# Frames in flight at N = 1 (the current stream as one render stream): D = 2 vs 3, alternating.
set -o pipefail
tag=${1:-r5n}
mkdir -p gpurun_out
for r in 1 2 3; do
  for p in 2 3; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --pipeline $p > gpurun_out/${tag}_p${p}_$r.json 2>/dev/null || exit 1
    python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read())
print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['frame_sha256'][:12])" gpurun_out/${tag}_p${p}_$r.json p$p
  done
done
for r in 1 2; do
  for p in 2 3; do
    timeout -k 10 200 python bench.py --no-cpu-baseline --steps 20 --warmup 5 --pipeline $p --scene scenes/utah-teapot-scene.json > gpurun_out/${tag}_c4p${p}_$r.json 2>/dev/null || exit 1
    python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read())
print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" gpurun_out/${tag}_c4p${p}_$r.json c4p$p
  done
done
