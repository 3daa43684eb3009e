# C4 under the max-ILP scheduler: shading threshold (NRT_WAVE_WAIT) 16 / 20 / 24 / 32, group fetch-ahead.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 1000 python scripts/ab_configs.py --reps 2 --steps 3 --out gpurun_out/r4v_ab.jsonl \
  --env ww24="" --env ww16="NRT_WAVE_WAIT=16" --env ww20="NRT_WAVE_WAIT=20" --env ww28="NRT_WAVE_WAIT=28" --env ww32="NRT_WAVE_WAIT=32" \
  --cfg c4="--scene scenes/utah-teapot-scene.json" || exit 1
echo r4v done
