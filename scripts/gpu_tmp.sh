# scratch GPU script (varies per experiment): library variants, bench + WRITE_SIZE each
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for v in default nr-ray-tracer_amd/build/w5/libnrt.so; do
  tag=$(basename $(dirname $v))
  if [ $v != default ]; then export NRT_LIB=$PWD/$v; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/t_$tag.json 2>gpurun_out/t_$tag.err || { tail -3 gpurun_out/t_$tag.err; exit 1; }
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/t_w$tag -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 > /dev/null 2>gpurun_out/t_w$tag.err || { tail -3 gpurun_out/t_w$tag.err; exit 1; }
  python3 - $tag <<'PY'
import csv, json, sys
t = sys.argv[1]
d = json.load(open(f"gpurun_out/t_{t}.json"))
tot = 0.0; n = set()
for r in csv.DictReader(open(f"gpurun_out/t_w{t}/run_counter_collection.csv")):
    if "render_kernel" in r["Kernel_Name"]:
        tot += float(r["Counter_Value"]); n.add(r["Dispatch_Id"])
print(t, d["value"], "Msamples/s", d["roofline"]["kernel_ms"], "ms  WRITE_SIZE/dispatch", tot / max(len(n), 1) * 1024)
PY
done
