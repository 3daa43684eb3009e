# scratch GPU script: WRITE_SIZE vs the Philox group size (NRT_WAVE_PIXELS)
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
for wp in 4 8 32; do
  export NRT_WAVE_PIXELS=$wp
  timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/w_$wp.json 2>/dev/null || exit 1
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('P', sys.argv[2], d['value'], d['roofline']['kernel_ms'])" gpurun_out/w_$wp.json $wp
  timeout -s KILL 90 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/wpmc_$wp -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 > /dev/null 2>&1 || exit 1
  python3 - gpurun_out/wpmc_$wp <<'PY'
import csv, glob, sys
rows = list(csv.DictReader(open(glob.glob(sys.argv[1] + "/**/run_counter_collection.csv", recursive=True)[0])))
v = [float(r["Counter_Value"]) for r in rows if "render_kernel" in r["Kernel_Name"]]
print("  WRITE_SIZE per dispatch (KB):", [round(x) for x in v][:4])
PY
done
