# C4 timing with and without rocprofv3 kernel tracing, same box, alternating.
set -o pipefail
tag=${1:-r5l}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
show() { python3 -c "
import json,sys
d=json.loads([l for l in open(sys.argv[1]) if l.startswith('{')][-1])
print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'])" $1 $2; }
for r in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --scene scenes/utah-teapot-scene.json --steps 20 > gpurun_out/${tag}_plain_$r.json 2>/dev/null || exit 1
  show gpurun_out/${tag}_plain_$r.json plain
  timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/${tag}_tr$r -o run --output-format csv -- python3 bench.py --no-cpu-baseline --scene scenes/utah-teapot-scene.json --steps 20 > gpurun_out/${tag}_trace_$r.json 2>/dev/null || exit 1
  show gpurun_out/${tag}_trace_$r.json traced
  timeout -k 10 200 python bench.py --no-cpu-baseline --scene scenes/utah-teapot-scene.json --steps 20 --pipeline 1 > gpurun_out/${tag}_p1_$r.json 2>/dev/null || exit 1
  show gpurun_out/${tag}_p1_$r.json pipeline1
done
