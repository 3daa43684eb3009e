# Claim staging with 16 slots per wave: timing against the previous build, WRITE_SIZE (earth f64).
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "f64 or exact or chacha or earth" > gpurun_out/r4q_pytest.log 2>&1 || { tail -30 gpurun_out/r4q_pytest.log; exit 1; }
tail -2 gpurun_out/r4q_pytest.log
C3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 16 --precision f64 --rng chacha8"
timeout -k 10 400 python scripts/ab_configs.py --reps 2 --steps 2 --out gpurun_out/r4q_ab.jsonl \
  --lib stg16=nr-ray-tracer_amd/nrt/libnrt.so --lib base=nr-ray-tracer_amd/ab/base/libnrt.so --cfg c3f64="$C3" || exit 1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r4q_w -o run --output-format csv -- python3 bench.py --no-cpu-baseline --kernel-only --steps 2 --warmup 1 $C3 > gpurun_out/r4q_w.json 2> gpurun_out/r4q_w.err || { echo "pmc failed"; exit 1; }
echo r4q done
