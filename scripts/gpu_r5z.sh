# Full GPU suite with the persistent exact walk as the default, then its threshold on the teapot.
set -o pipefail
tag=${1:-r5z}
bash scripts/gpu_full.sh $tag || exit 1
timeout -k 10 600 python scripts/ab_configs.py --reps 2 --steps 4 --timeout 200 --out gpurun_out/${tag}_ab.jsonl \
  --env dflt="" --env p40="NRT_WAVE_WAIT=40" --env p44="NRT_WAVE_WAIT=44" \
  --cfg c4f64="--precision f64 --rng chacha8 --scene scenes/utah-teapot-scene.json"
