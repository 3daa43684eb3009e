# C4 node decode variants on the round-4 trips: v_perm + v_fma_mix plane bytes (NRT_NODE_MIX),
# packed (near, far) slab pairs (NRT_PK_SLAB).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 900 python scripts/ab_configs.py --reps 3 --steps 3 --out gpurun_out/r4n_ab.jsonl \
  --env base="" --env mix="NRT_JIT_DEFS=-DNRT_NODE_MIX=1" --env pk="NRT_JIT_DEFS=-DNRT_PK_SLAB=1" \
  --cfg c4="--scene scenes/utah-teapot-scene.json" || exit 1
echo r4n done
