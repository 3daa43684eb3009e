set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4e_pytest.log 2>&1 || { tail -30 gpurun_out/r4e_pytest.log; exit 1; }
tail -1 gpurun_out/r4e_pytest.log
timeout -k 10 600 python scripts/ab_configs.py --reps 2 --out gpurun_out/r4e_ab.jsonl --lib A=nr-ray-tracer_amd/ab/on1/libnrt.so --lib B=nr-ray-tracer_amd/nrt/libnrt.so \
  --cfg c3f64="--scene scenes/earth.toml --width 1920 --height 1080 --spp 16 --precision f64 --rng chacha8" \
  --cfg c5f64="--spp 64 --precision f64 --rng chacha8" --cfg c4f64="--scene scenes/utah-teapot-scene.json --spp 16 --precision f64 --rng chacha8" 2>&1 | tail -4 || exit 1
for c in WRITE_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c -d gpurun_out/r4e_pmc_$c -o run --output-format csv -- python3 bench.py --no-cpu-baseline --kernel-only --steps 2 --warmup 1 --scene scenes/earth.toml --width 1920 --height 1080 --spp 16 --precision f64 --rng chacha8 > /dev/null 2> gpurun_out/r4e_pmc_$c.err || { echo "pmc $c failed"; tail -3 gpurun_out/r4e_pmc_$c.err; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/r4e_pmc_$c --json gpurun_out/r4e_pmc_$c.json > /dev/null
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['hbm_write_bytes'])" gpurun_out/r4e_pmc_$c.json $c
done
