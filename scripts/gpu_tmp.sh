set -o pipefail
for env in "X=1" "NRT_SAH_PRIM_COST=0.34" "NRT_SAH_PRIM_COST=0.67" "NRT_SAH_PRIM_COST=2" "NRT_WBVH4=0"; do
  env $env timeout -k 10 120 python bench.py --no-cpu-baseline --precision f64 --rng chacha8 --steps 1 --warmup 1 > /tmp/l.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('/tmp/l.json')); print('$env', d['value'], d['timings_ms']['kernel_device_only'], d['frame_sha256'][:16])"
done
