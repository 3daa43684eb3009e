set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/x_pytest.log 2>&1 || { tail -30 gpurun_out/x_pytest.log; exit 1; }
tail -2 gpurun_out/x_pytest.log
for i in 1 2; do for lib in nr-ray-tracer_amd/ab/base.so nr-ray-tracer_amd/nrt/libnrt.so; do
  for sc in scenes/cornell-box-scene.json scenes/utah-teapot-scene.json; do
  NRT_LIB=$PWD/$lib timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --precision f64 --rng chacha8 --scene $sc > gpurun_out/x.json 2> gpurun_out/x.err || { echo fail; tail -3 gpurun_out/x.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], sys.argv[3][7:20], d['value'], d['timings_ms']['kernel_device_only'], d['frame_sha256'][:12])" gpurun_out/x.json $lib $sc
done; done; done
