# Ad-hoc GPU experiment of the current round (edited per experiment; see scripts/ab_configs.py).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
tag=${1:-e7}
timeout -k 10 600 python -u -m pytest tests -m gpu -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1; tail -3 gpurun_out/${tag}_pytest.log
C4="--scene scenes/utah-teapot-scene.json"; C3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 128"; C1B="--scene scenes/spheres.toml --width 1920 --height 1080 --spp 64"
AB="timeout -k 10 900 python scripts/ab_configs.py --reps 2"
NEW=nr-ray-tracer_amd/nrt/libnrt.so
$AB --out gpurun_out/${tag}_sph.jsonl --lib base=nr-ray-tracer_amd/ab/base/libnrt.so --lib new=$NEW --env def="" --env s64="NRT_SPHERE_F32=0" --env all32="NRT_SPHERE_F32=2" --env all32np="NRT_SPHERE_F32=2 NRT_JIT_DEFS=-DNRT_SPHERE_REPROJ=0" --env noproj="NRT_JIT_DEFS=-DNRT_SPHERE_REPROJ=0" \
  --cfg c3="$C3" --cfg c1b="$C1B" || exit 1
$AB --out gpurun_out/${tag}_c5.jsonl --lib base=nr-ray-tracer_amd/ab/base/libnrt.so --lib new=$NEW --cfg c5="" --cfg c5x="--precision f64 --rng chacha8 --spp 64" || exit 1
pmc() {  # name lib env counter bench-args...
  local n=$1 lib=$2 ev=$3 c=$4; shift 4
  env NRT_LIB=$PWD/$lib $ev timeout -s KILL 120 rocprofv3 --pmc $c -d gpurun_out/${tag}_pmc_$n -o run --output-format csv -- python3 bench.py --no-cpu-baseline --kernel-only --steps 2 --warmup 1 "$@" > /dev/null 2> gpurun_out/${tag}_pmc_$n.err || { echo "pmc $n failed"; tail -3 gpurun_out/${tag}_pmc_$n.err; exit 1; }
}
pmc c5l $NEW "" "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_LDS"
echo done
