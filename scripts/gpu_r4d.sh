set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4d_pytest.log 2>&1 || { tail -30 gpurun_out/r4d_pytest.log; exit 1; }
tail -1 gpurun_out/r4d_pytest.log
timeout -k 10 120 python scripts/shard_timing.py > gpurun_out/r4d_shard.json && cat gpurun_out/r4d_shard.json
NRT_WAVE_PIXELS=1 timeout -k 10 120 python scripts/shard_timing.py scenes/cornell-box-scene.json 1024 1024 256 1,4,8 && \
timeout -k 10 300 python scripts/ab_configs.py --reps 2 --out gpurun_out/r4d_ab.jsonl --lib A=nr-ray-tracer_amd/ab/on1/libnrt.so --lib B=nr-ray-tracer_amd/nrt/libnrt.so --cfg c3f64="--scene scenes/earth.toml --width 1920 --height 1080 --spp 16 --precision f64 --rng chacha8" 2>&1 | tail -3 && \
for c in WRITE_SIZE FETCH_SIZE; do
  timeout -s KILL 90 rocprofv3 --pmc $c -d gpurun_out/r4d_pmc_$c -o run --output-format csv -- python3 bench.py --no-cpu-baseline --kernel-only --steps 2 --warmup 1 --scene scenes/earth.toml --width 1920 --height 1080 --spp 16 --precision f64 --rng chacha8 > /dev/null 2> gpurun_out/r4d_pmc_$c.err || { echo "pmc $c failed"; tail -3 gpurun_out/r4d_pmc_$c.err; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/r4d_pmc_$c --json gpurun_out/r4d_pmc_$c.json > /dev/null
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['per_dispatch'].get(sys.argv[2]))" gpurun_out/r4d_pmc_$c.json $c
done
