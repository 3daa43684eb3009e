set -o pipefail
mkdir -p gpurun_out
timeout -k 10 200 python -u -m pytest tests/test_gpu_parity.py -k "specialised" -x -q --timeout 120 --timeout-method thread > gpurun_out/j_pytest.log 2>&1 || { tail -30 gpurun_out/j_pytest.log; exit 1; }
tail -2 gpurun_out/j_pytest.log
for sc in scenes/utah-teapot-scene.json; do
for j in 0 1 0 1; do
  NRT_JIT=$j timeout -k 10 120 python bench.py --steps 3 --warmup 1 --no-cpu-baseline --rng chacha8 --scene $sc > gpurun_out/j.json 2> gpurun_out/j.err || { echo fail; tail -3 gpurun_out/j.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], 'jit', sys.argv[3], d['value'], d['timings_ms']['kernel_device_only'], d['frame_sha256'][:12], d.get('jit'))" gpurun_out/j.json $sc $j
done; done
