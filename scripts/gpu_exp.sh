# Ad-hoc GPU experiment of the current round (edited per experiment; see scripts/ab_configs.py).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
tag=${1:-e6}
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1; tail -5 gpurun_out/${tag}_pytest.log
C4="--scene scenes/utah-teapot-scene.json"; C3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 128"
AB="timeout -k 10 900 python scripts/ab_configs.py --reps 2"
NEW=nr-ray-tracer_amd/nrt/libnrt.so
$AB --out gpurun_out/${tag}_ab.jsonl --lib base=nr-ray-tracer_amd/ab/base/libnrt.so --lib new=$NEW \
  --cfg c5="" --cfg c4="$C4" --cfg c3="$C3" --cfg c1b="--scene scenes/spheres.toml --width 1920 --height 1080 --spp 64" \
  --cfg c5x="--precision f64 --rng chacha8 --spp 64" --cfg c4x="$C4 --precision f64 --rng chacha8 --spp 64" || exit 1
$AB --out gpurun_out/${tag}_grab.jsonl --lib new=$NEW --env g1="" --env g2="NRT_JIT_DEFS=-DNRT_GRAB=2" --env g4="NRT_JIT_DEFS=-DNRT_GRAB=4" \
  --cfg c5="" --cfg c4="$C4" --cfg c3="$C3" || exit 1
$AB --out gpurun_out/${tag}_knobs.jsonl --lib new=$NEW --env def="" --env nocomp="NRT_WBVH_COMPACT=0" --env leaf8="NRT_WBVH_LEAF=8 NRT_WBVH_COMPACT=0" --cfg c4="$C4" || exit 1
$AB --out gpurun_out/${tag}_knobs.jsonl --lib new=$NEW --env def="" --env stackwalk="NRT_EXACT_THREAD=0" \
  --cfg c5x="--precision f64 --rng chacha8 --spp 64" --cfg c4x="$C4 --precision f64 --rng chacha8 --spp 64" || exit 1
$AB --out gpurun_out/${tag}_tex.jsonl --lib new=$NEW --cfg c3="$C3" || exit 1
$AB --out gpurun_out/${tag}_tex.jsonl --lib rowmajor=nr-ray-tracer_amd/ab/rowmajor/libnrt.so --env rm="NRT_JIT_DEFS=-DNRT_TEX_ROWMAJOR" --cfg c3="$C3" || exit 1
pmc() {  # name lib env counter bench-args...
  local n=$1 lib=$2 ev=$3 c=$4; shift 4
  env NRT_LIB=$PWD/$lib $ev timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/${tag}_pmc_$n -o run --output-format csv -- python3 bench.py --no-cpu-baseline --kernel-only --steps 2 --warmup 1 "$@" > /dev/null 2> gpurun_out/${tag}_pmc_$n.err || { echo "pmc $n failed"; tail -3 gpurun_out/${tag}_pmc_$n.err; exit 1; }
}
pmc c5w_g1 $NEW "" WRITE_SIZE
pmc c5w_g4 $NEW "NRT_JIT_DEFS=-DNRT_GRAB=4" WRITE_SIZE
pmc c3f_new $NEW "" FETCH_SIZE $C3
pmc c3f_row nr-ray-tracer_amd/ab/rowmajor/libnrt.so "NRT_JIT_DEFS=-DNRT_TEX_ROWMAJOR" FETCH_SIZE $C3
pmc c5xw_new $NEW "" WRITE_SIZE --precision f64 --rng chacha8 --spp 64
pmc c4xw_new $NEW "" WRITE_SIZE $C4 --precision f64 --rng chacha8 --spp 64
echo done
