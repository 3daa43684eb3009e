# C4 under the max-ILP scheduler: waves per SIMD (launch bounds) 5 / 6 / 7.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 800 python scripts/ab_configs.py --reps 2 --steps 3 --out gpurun_out/r4u_ab.jsonl \
  --env w6="" --env w5="NRT_JIT_DEFS=-DNRT_WBVH_WAVES=5" --env w7="NRT_JIT_DEFS=-DNRT_WBVH_WAVES=7" \
  --cfg c4="--scene scenes/utah-teapot-scene.json" || exit 1
echo r4u done
