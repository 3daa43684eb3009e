# Headline evidence for the final library: C5 (default, pipelined) and C5 without overlap profiled
# (kernel trace + PMC passes), then the f32 configs whose kernels changed (C5, C4, C3) benched.
# usage: bash scripts/gpu_headline.sh <tag>;  then python scripts/publish_profiles.py <tag> --as r06
set -o pipefail
tag=${1:-r6z}
mkdir -p gpurun_out
bash scripts/profile.sh ${tag}_c5_f32_philox --steps 20 --warmup 2 > gpurun_out/${tag}_prof_c5.log 2>&1 || { tail -5 gpurun_out/${tag}_prof_c5.log; exit 1; }
tail -1 gpurun_out/${tag}_prof_c5.log
bash scripts/profile.sh ${tag}_c5_f32_philox_pipeline0 --pipeline 1 --steps 20 --warmup 2 > gpurun_out/${tag}_prof_c5p0.log 2>&1 || { tail -5 gpurun_out/${tag}_prof_c5p0.log; exit 1; }
tail -1 gpurun_out/${tag}_prof_c5p0.log
run() {  # name, args...
  local name=$1; shift
  timeout -k 10 300 python bench.py --steps 20 --warmup 2 --no-cpu-baseline "$@" > gpurun_out/${tag}_cfg_$name.json 2> gpurun_out/${tag}_cfg_$name.err || { echo "bench $name failed rc=$?"; tail -3 gpurun_out/${tag}_cfg_$name.err; return 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Msamples/s', d['roofline']['kernel_ms'], 'ms')" gpurun_out/${tag}_cfg_$name.json $name
}
run c5_f32 && run c4_f32 --scene scenes/utah-teapot-scene.json && \
run c3_f32 --scene scenes/earth.toml --width 1920 --height 1080 --spp 128 && run c5_f32_b && \
run c2_f32 --scene scenes/cornell-box-scene.json --width 512 --height 512 --spp 64
