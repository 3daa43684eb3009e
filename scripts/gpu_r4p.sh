# Claim staging in the persistent lanes (coalesced writes of a claim's pixels): exact / ChaCha8
# parity tests, alternating timing against the previous build, WRITE_SIZE of the earth f64 launch.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4p_pytest.log 2>&1 || { tail -30 gpurun_out/r4p_pytest.log; exit 1; }
tail -2 gpurun_out/r4p_pytest.log
C3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 16 --precision f64 --rng chacha8"
timeout -k 10 600 python scripts/ab_configs.py --reps 2 --steps 2 --out gpurun_out/r4p_ab.jsonl \
  --lib stg=nr-ray-tracer_amd/nrt/libnrt.so --lib base=nr-ray-tracer_amd/ab/base/libnrt.so \
  --cfg c3f64="$C3" --cfg c3f64s8="--scene scenes/earth.toml --width 1920 --height 1080 --spp 8 --precision f64 --rng chacha8" \
  --cfg c2f64="--scene scenes/cornell-box-scene.json --width 512 --height 512 --spp 64 --precision f64 --rng chacha8" || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r4p_w -o run --output-format csv -- python3 bench.py --no-cpu-baseline --kernel-only --steps 2 --warmup 1 $C3 > gpurun_out/r4p_w.json 2> gpurun_out/r4p_w.err || { echo "pmc failed"; exit 1; }
echo r4p done
