# VALU instructions per launch of the headline kernel with one vs two groups per queue atomic (same box).
set -o pipefail
cd /tmp && export TMPDIR=/tmp && cd - > /dev/null
for g in 2 1; do
  rm -rf gpurun_out/r5bl_g$g
  NRT_JIT_DEFS="-DNRT_GRAB_FLAT=$g" timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_WAVES SQ_INSTS_SALU -d gpurun_out/r5bl_g$g -o run --output-format csv -- python3 bench.py --no-cpu-baseline --kernel-only --steps 4 --warmup 1 > gpurun_out/r5bl_g$g.json 2> gpurun_out/r5bl_g$g.err || { tail -3 gpurun_out/r5bl_g$g.err; exit 1; }
  python3 - gpurun_out/r5bl_g$g <<'PY'
import csv, glob, sys, collections
f = glob.glob(sys.argv[1] + "/**/*counter_collection.csv", recursive=True)[0]
acc = collections.defaultdict(lambda: collections.defaultdict(float))
for r in csv.DictReader(open(f)):
    if "render_kernel" not in r["Kernel_Name"]:
        continue
    acc[r["Dispatch_Id"]][r["Counter_Name"]] += float(r["Counter_Value"])
vals = sorted(v["SQ_INSTS_VALU"] for v in acc.values())
print(sys.argv[1], "dispatches", len(vals), "VALU per dispatch", ["%.3g" % v for v in vals])
PY
done
