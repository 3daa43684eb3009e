# HBM traffic attribution of one kernel variant: FETCH_SIZE / WRITE_SIZE per launch (separate PMC passes,
# MI355X_MICROARCH.md's FETCH x2 correction in pmc_summary.py) at several spp, so per-pixel traffic
# (framebuffer, pixel-claim atomics) and per-sample traffic (tree / texel reads, spills) separate.
# usage: bash scripts/traffic_attrib.sh <tag> "<spp list>" <bench args...>   (env knobs pass through)
set -o pipefail
tag=$1; spps=$2; shift 2
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/ta_$tag
for spp in $spps; do
  for c in FETCH_SIZE WRITE_SIZE; do
    d=gpurun_out/ta_$tag/spp${spp}_$c
    timeout -s KILL 120 rocprofv3 --pmc $c -d $d -o run --output-format csv -- python3 bench.py --no-cpu-baseline --kernel-only --steps 2 --warmup 1 --spp $spp "$@" > $d.json 2> $d.err || { echo "pass $spp $c failed"; tail -3 $d.err; exit 1; }
    python3 scripts/pmc_summary.py $d --json $d.sum.json > /dev/null || exit 1
  done
  python3 - "$tag" "$spp" <<'PY'
import json, sys
t, spp = sys.argv[1], sys.argv[2]
f = json.load(open(f"gpurun_out/ta_{t}/spp{spp}_FETCH_SIZE.sum.json"))
w = json.load(open(f"gpurun_out/ta_{t}/spp{spp}_WRITE_SIZE.sum.json"))
b = json.loads(open(f"gpurun_out/ta_{t}/spp{spp}_FETCH_SIZE.json").read().strip().splitlines()[-1])
print(json.dumps({"tag": t, "spp": int(spp), "fetch_bytes": f.get("hbm_fetch_bytes"), "write_bytes": w.get("hbm_write_bytes"),
                  "kernel_ms": b["roofline"]["kernel_ms"], "config": b["config"]["workload"]}))
PY
done
