# Round-4 GPU batch: GPU suite, default bench line, then the A/B experiments (alternating runs).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4g_pytest.log 2>&1 || { tail -30 gpurun_out/r4g_pytest.log; exit 1; }
tail -1 gpurun_out/r4g_pytest.log
<<<<<<< HEAD
timeout -k 10 200 python bench.py > gpurun_out/r4g_bench.json 2> gpurun_out/r4g_bench.err || { tail -5 gpurun_out/r4g_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4g_bench.json')); print('bench', d['value'], d['timings_ms'], d['kernel_variant'])"
ab() { timeout -k 10 900 python scripts/ab_configs.py --reps 2 --lib B=nr-ray-tracer_amd/nrt/libnrt.so "$@" 2>&1 | tail -12; }
ab --out gpurun_out/r4g_ab_tail.jsonl --env t1="NRT_TAIL=1" --env t0="NRT_TAIL=0" --cfg c5="" --cfg c4="--scene scenes/utah-teapot-scene.json" --cfg c3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 128" || exit 1
timeout -k 10 120 python scripts/shard_timing.py > gpurun_out/r4g_shard_tail1.json && cat gpurun_out/r4g_shard_tail1.json || exit 1
NRT_TAIL=0 timeout -k 10 120 python scripts/shard_timing.py > gpurun_out/r4g_shard_tail0.json && cat gpurun_out/r4g_shard_tail0.json || exit 1
ab --out gpurun_out/r4g_ab_c5cam.jsonl --env base="NRT_JIT_DEFS=" --env cam7="NRT_JIT_DEFS=-DNRT_CAMF_AT_USE=1" --env cam8="NRT_JIT_DEFS=-DNRT_CAMF_AT_USE=1 -DNRT_WORLD_LIST_WAVES=8" --env w8="NRT_JIT_DEFS=-DNRT_WORLD_LIST_WAVES=8" --cfg c5="" || exit 1
ab --out gpurun_out/r4g_ab_c4pf.jsonl --env base="NRT_JIT_DEFS=" --env pf6="NRT_JIT_DEFS=-DNRT_NODE_PREFETCH=1" --env pf5="NRT_JIT_DEFS=-DNRT_NODE_PREFETCH=1 -DNRT_WBVH_WAVES=5" \
  --env pp6="NRT_JIT_DEFS=-DNRT_PRIM_PREFETCH=1" --env both5="NRT_JIT_DEFS=-DNRT_PRIM_PREFETCH=1 -DNRT_NODE_PREFETCH=1 -DNRT_WBVH_WAVES=5" --cfg c4="--scene scenes/utah-teapot-scene.json" || exit 1
ab --out gpurun_out/r4g_abpal.jsonl --env pal1="NRT_TEX_PAL=1" --env pal0="NRT_TEX_PAL=0" --cfg c3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 128" || exit 1
=======
timeout -k 10 600 python scripts/ab_configs.py --reps 3 --out gpurun_out/r4g_abpal.jsonl --lib B=nr-ray-tracer_amd/nrt/libnrt.so --env pal1="NRT_TEX_PAL=1" --env pal0="NRT_TEX_PAL=0" \
  --cfg c3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 128" 2>&1 | tail -3 || exit 1
timeout -k 10 300 python scripts/ab_configs.py --reps 2 --out gpurun_out/r4g_ab.jsonl --lib A=nr-ray-tracer_amd/ab/on1/libnrt.so --lib B=nr-ray-tracer_amd/nrt/libnrt.so --cfg c5="" --cfg c2="--scene scenes/cornell-box-scene.json --width 512 --height 512 --spp 64" 2>&1 | tail -5 || exit 1
timeout -k 10 200 python bench.py > gpurun_out/r4g_bench.json 2> gpurun_out/r4g_bench.err && cat gpurun_out/r4g_bench.json | head -c 600
timeout -k 10 700 python scripts/ab_configs.py --reps 2 --out gpurun_out/r4h_ab_c4.jsonl --lib B=nr-ray-tracer_amd/nrt/libnrt.so \
  --env base="NRT_JIT_DEFS=" --env pf6="NRT_JIT_DEFS=-DNRT_NODE_PREFETCH=1" --env pf5="NRT_JIT_DEFS=-DNRT_NODE_PREFETCH=1 -DNRT_WBVH_WAVES=5" \
  --cfg c4="--scene scenes/utah-teapot-scene.json" 2>&1 | tail -4 || exit 1
timeout -k 10 400 python scripts/ab_configs.py --reps 2 --out gpurun_out/r4h_ab_c5.jsonl --lib B=nr-ray-tracer_amd/nrt/libnrt.so \
  --env w6="NRT_JIT_DEFS=" --env w8="NRT_JIT_DEFS=-DNRT_WORLD_LIST_WAVES=8" --env w7="NRT_JIT_DEFS=-DNRT_WORLD_LIST_WAVES=7" \
  --cfg c5="" 2>&1 | tail -4 || exit 1
>>>>>>> parent of ee60b86 (If-if trips: optional leaf-primitive prefetch (NRT_PRIM_PREFETCH, off; A/B pending))
