# scratch GPU script (varies per experiment): GPU tests, C4 / C1-big / C5 benches
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_pytest.log 2>&1 || { tail -30 gpurun_out/t_pytest.log; exit 1; }
tail -2 gpurun_out/t_pytest.log
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/t_$name.json 2> gpurun_out/t_$name.err || { echo "bench $name failed rc=$?"; tail -3 gpurun_out/t_$name.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Msamples/s', d['roofline']['kernel_ms'], 'ms')" gpurun_out/t_$name.json $name
}
run c4_f32 --scene scenes/utah-teapot-scene.json && run c1_f32_big --scene scenes/spheres.toml --width 1920 --height 1080 --spp 64 && run c5_f32
