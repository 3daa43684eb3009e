# Alternating A/B bench runs of one config: arm A = the tree as is, arm B = the same with an env
# assignment (e.g. NRT_EXACT_CLAIM=1).  usage: bash scripts/ab_quick.sh <tag> <reps> "<B env>" <bench args...>
set -o pipefail
tag=$1; reps=$2; benv=$3; shift 3
mkdir -p gpurun_out
for k in $(seq 1 $reps); do
  timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/${tag}_A_$k.json 2> gpurun_out/${tag}_A_$k.err || { tail -3 gpurun_out/${tag}_A_$k.err; exit 1; }
  env $benv timeout -k 10 300 python bench.py --no-cpu-baseline "$@" > gpurun_out/${tag}_B_$k.json 2> gpurun_out/${tag}_B_$k.err || { tail -3 gpurun_out/${tag}_B_$k.err; exit 1; }
done
python3 - "$tag" <<'PY'
import glob, json, sys
t = sys.argv[1]
for arm in "AB":
    for f in sorted(glob.glob(f"gpurun_out/{t}_{arm}_*.json")):
        d = json.loads(open(f).read().strip().splitlines()[-1])
        print(t, arm, d["value"], d["ms_per_step"], d["roofline"]["kernel_ms"], (d.get("frame_sha256") or "")[:12], d["kernel_variant"])
PY
