set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4f_pytest.log 2>&1 || { tail -30 gpurun_out/r4f_pytest.log; exit 1; }
tail -1 gpurun_out/r4f_pytest.log
rm -f gpurun_out/r4f_jit_dump.txt
NRT_JIT_DUMP=gpurun_out/r4f_jit_dump.txt timeout -k 10 100 python bench.py --steps 1 --warmup 1 --no-cpu-baseline > /dev/null || exit 1
NRT_JIT_DUMP=gpurun_out/r4f_jit_dump.txt timeout -k 10 100 python bench.py --steps 1 --warmup 1 --no-cpu-baseline --scene scenes/earth.toml --width 1920 --height 1080 --spp 128 > /dev/null || exit 1
timeout -k 10 600 python scripts/ab_configs.py --reps 2 --out gpurun_out/r4f_ab.jsonl --lib B=nr-ray-tracer_amd/nrt/libnrt.so --env rec1="NRT_JIT_RECORDS=1" --env rec0="NRT_JIT_RECORDS=0" \
  --cfg c5="" --cfg c3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 128" --cfg c2="--scene scenes/cornell-box-scene.json --width 512 --height 512 --spp 64" 2>&1 | tail -7 || exit 1
timeout -k 10 600 python scripts/ab_configs.py --reps 2 --out gpurun_out/r4f_ab64.jsonl --lib A=nr-ray-tracer_amd/ab/on1/libnrt.so --lib B=nr-ray-tracer_amd/nrt/libnrt.so \
  --cfg c3f64="--scene scenes/earth.toml --width 1920 --height 1080 --spp 16 --precision f64 --rng chacha8" \
  --cfg c5f64="--spp 64 --precision f64 --rng chacha8" --cfg c4f64="--scene scenes/utah-teapot-scene.json --spp 16 --precision f64 --rng chacha8" 2>&1 | tail -7 || exit 1
for c in WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c -d gpurun_out/r4f_pmc_$c -o run --output-format csv -- python3 bench.py --no-cpu-baseline --kernel-only --steps 2 --warmup 1 --scene scenes/earth.toml --width 1920 --height 1080 --spp 16 --precision f64 --rng chacha8 > /dev/null 2> gpurun_out/r4f_pmc_$c.err || { echo "pmc $c failed"; tail -3 gpurun_out/r4f_pmc_$c.err; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/r4f_pmc_$c --json gpurun_out/r4f_pmc_$c.json > /dev/null
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['hbm_write_bytes'])" gpurun_out/r4f_pmc_$c.json $c
done
timeout -k 10 600 python scripts/ab_configs.py --reps 2 --out gpurun_out/r4f_abpal.jsonl --lib B=nr-ray-tracer_amd/nrt/libnrt.so --env pal1="NRT_TEX_PAL=1" --env pal0="NRT_TEX_PAL=0" \
  --cfg c3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 128" 2>&1 | tail -3 || exit 1
for pal in 1 0; do
  NRT_TEX_PAL=$pal timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/r4f_pmc_fetch_pal$pal -o run --output-format csv -- python3 bench.py --no-cpu-baseline --kernel-only --steps 2 --warmup 1 --scene scenes/earth.toml --width 1920 --height 1080 --spp 128 > /dev/null 2> gpurun_out/r4f_pmc_fetch_pal$pal.err || { echo "pmc fetch failed"; tail -3 gpurun_out/r4f_pmc_fetch_pal$pal.err; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/r4f_pmc_fetch_pal$pal --json gpurun_out/r4f_pmc_fetch_pal$pal.json > /dev/null
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('pal', sys.argv[2], 'FETCH', d['hbm_fetch_bytes'])" gpurun_out/r4f_pmc_fetch_pal$pal.json $pal
done
