# Quick GPU iteration: GPU test suite, default bench line, one WRITE_SIZE/FETCH_SIZE PMC pass each.
# usage: bash scripts/gpu_quick.sh <tag> [bench args...]
set -o pipefail
tag=${1:-q}; shift
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest.log
timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/${tag}_bench.json 2> gpurun_out/${tag}_bench.err || { tail -5 gpurun_out/${tag}_bench.err; exit 1; }
cat gpurun_out/${tag}_bench.json
for c in WRITE_SIZE FETCH_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c -d gpurun_out/${tag}_pmc_$c -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 "$@" > /dev/null 2> gpurun_out/${tag}_pmc_$c.err || { echo "pmc $c failed"; tail -3 gpurun_out/${tag}_pmc_$c.err; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/${tag}_pmc_$c --json gpurun_out/${tag}_pmc_$c.json > /dev/null
done
python3 - "$tag" <<'PY'
import json, sys, glob
t = sys.argv[1]
for c in ("WRITE_SIZE", "FETCH_SIZE"):
    try:
        d = json.load(open(f"gpurun_out/{t}_pmc_{c}.json"))
        print(c, d["per_dispatch"].get(c), "KiB/dispatch")
    except Exception as e:
        print(c, "n/a", e)
PY
