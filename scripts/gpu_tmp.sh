set -o pipefail
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 200 --timeout-method thread -k "specialised or stat or philox" > gpurun_out/gputest_jit.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -4 gpurun_out/gputest_jit.log; [ $rc = 0 ] || exit 1
for i in 1 2; do for jit in 0 1; do
  for args in "--scene scenes/utah-teapot-scene.json --steps 3 --warmup 1" "--scene scenes/spheres.toml --width 1920 --height 1080 --spp 64 --steps 3 --warmup 1"; do
  NRT_JIT=$jit timeout -k 10 120 python bench.py --no-cpu-baseline $args > /tmp/l.json 2>/dev/null || exit 1
  python -c "import json; d=json.load(open('/tmp/l.json')); print('jit=$jit', d['config']['workload'], d['value'], d['timings_ms']['kernel_device_only'], d['jit'])"
done; done; done
