set -o pipefail
NRT_SPLIT=4 timeout -k 10 600 python -m pytest tests -m gpu -q -k "philox or statistically" > gpurun_out/r1split_pytest.log 2>&1; tail -2 gpurun_out/r1split_pytest.log
for sp in 1 2 4 8; do
  for h in 1024 128; do
    NRT_SPLIT=$sp timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --height $h > gpurun_out/sp.json 2>gpurun_out/sp.err || { echo fail; tail -3 gpurun_out/sp.err; exit 1; }
    python3 -c "import json,sys; d=json.load(open('gpurun_out/sp.json')); print('split', sys.argv[1], 'rows', sys.argv[2], d['value'], d['roofline']['kernel_ms'])" $sp $h
  done
done
for sp in 1 4 8; do
  NRT_SPLIT=$sp timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --scene scenes/utah-teapot-scene.json > gpurun_out/sp.json 2>gpurun_out/sp.err || { echo fail; exit 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/sp.json')); print('teapot split', sys.argv[1], d['value'])" $sp
done
