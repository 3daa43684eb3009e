# Ad-hoc GPU experiment of the current round (edited per experiment; see scripts/ab_configs.py).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
tag=${1:-e8}
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -1 gpurun_out/${tag}_pytest.log
C4="--scene scenes/utah-teapot-scene.json"; C3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 128"; C1B="--scene scenes/spheres.toml --width 1920 --height 1080 --spp 64"
C5X="--precision f64 --rng chacha8 --spp 64"; C4X="$C4 --precision f64 --rng chacha8 --spp 16"
AB="timeout -k 10 900 python scripts/ab_configs.py --reps 2"
BASE=nr-ray-tracer_amd/ab/base/libnrt.so; NEW=nr-ray-tracer_amd/nrt/libnrt.so
$AB --out gpurun_out/${tag}_c4.jsonl --lib new=$NEW --env ww16="NRT_WAVE_WAIT=16" --env ww20="NRT_WAVE_WAIT=20" --env ww24="NRT_WAVE_WAIT=24" --env ww28="NRT_WAVE_WAIT=28" --env ww32="" --cfg c4="$C4" --cfg c1b="$C1B" || exit 1
$AB --out gpurun_out/${tag}_x.jsonl --lib new=$NEW --lib uni=nr-ray-tracer_amd/ab/uni/libnrt.so --cfg c5x="$C5X" --cfg c4x="$C4X" || exit 1
pmc() {  # name lib counters bench-args...
  local n=$1 lib=$2 c=$3; shift 3
  env NRT_LIB=$PWD/$lib timeout -s KILL 180 rocprofv3 --pmc $c -d gpurun_out/${tag}_pmc_$n -o run --output-format csv -- python3 bench.py --no-cpu-baseline --kernel-only --steps 2 --warmup 1 "$@" > /dev/null 2> gpurun_out/${tag}_pmc_$n.err || { echo "pmc $n failed"; tail -3 gpurun_out/${tag}_pmc_$n.err; exit 1; }
}
echo done
