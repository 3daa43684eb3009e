# GPU suite + full-frame JIT/generic comparison + alternating A/B of two library builds.
# usage: bash scripts/gpu_ab.sh <tag> <libA> <libB> [reps]   (libs relative to the repo root)
set -o pipefail
tag=${1:-ab}; a=$2; b=$3; reps=${4:-2}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest.log
timeout -k 10 120 python scripts/jit_compare.py > gpurun_out/${tag}_jit_compare.log 2>&1; rc=$?; cat gpurun_out/${tag}_jit_compare.log; [ $rc -le 1 ] || exit 1
timeout -k 10 900 python scripts/ab_configs.py --reps $reps --out gpurun_out/${tag}_ab.jsonl --lib A=$a --lib B=$b \
  --cfg c5="" --cfg c4="--scene scenes/utah-teapot-scene.json" \
  --cfg c3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 128" \
  --cfg c2="--scene scenes/cornell-box-scene.json --width 512 --height 512 --spp 64" || exit 1
