# scratch GPU script (varies per experiment)
set -o pipefail
mkdir -p gpurun_out
b() {  # tag, args
  local tag=$1; shift
  timeout -k 10 120 python bench.py --steps 2 --warmup 1 --no-cpu-baseline "$@" > gpurun_out/p6.json 2>gpurun_out/p6.err || { tail -3 gpurun_out/p6.err; return 1; }
  python3 -c "import json,sys; d=json.load(open('gpurun_out/p6.json')); print(sys.argv[1], d['value'], d['roofline']['kernel_ms'])" "$tag"
}
for ww in 1 4 16 32; do NRT_WAVE_WAIT=$ww b "c4 wait $ww" --scene scenes/utah-teapot-scene.json || exit 1; done
for wp in 1 2 8 16; do NRT_WAVE_PIXELS=$wp b "c4 wp $wp" --scene scenes/utah-teapot-scene.json || exit 1; done
for ww in 4 16 32; do NRT_WAVE_WAIT=$ww b "c1big wait $ww" --scene scenes/spheres.toml --width 1920 --height 1080 --spp 64 || exit 1; done
