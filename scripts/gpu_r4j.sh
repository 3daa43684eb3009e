# f64 persistent lanes: pixel claims of >= 8 per counter atomic (default build) vs 1 (ab/claim1):
# exact-kernel parity tests, alternating kernel timing, WRITE_SIZE per launch of both.
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread -k "f64 or exact or chacha" > gpurun_out/r4j_pytest.log 2>&1 || { tail -30 gpurun_out/r4j_pytest.log; exit 1; }
tail -2 gpurun_out/r4j_pytest.log
C3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 16 --precision f64 --rng chacha8"
C5="--precision f64 --rng chacha8"
C4="--scene scenes/utah-teapot-scene.json --precision f64 --rng chacha8"
timeout -k 10 600 python scripts/ab_configs.py --reps 2 --steps 2 --out gpurun_out/r4j_ab.jsonl \
  --lib claim8=nr-ray-tracer_amd/nrt/libnrt.so --lib claim1=nr-ray-tracer_amd/ab/claim1/libnrt.so \
  --cfg c3f64="$C3" --cfg c5f64="$C5" --cfg c4f64="$C4" || exit 1
for v in claim8:nr-ray-tracer_amd/nrt/libnrt.so claim1:nr-ray-tracer_amd/ab/claim1/libnrt.so; do
  n=${v%%:*}; l=${v#*:}
  NRT_LIB=$PWD/$l timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE -d gpurun_out/r4j_w_$n -o run --output-format csv -- python3 bench.py --no-cpu-baseline --kernel-only --steps 2 --warmup 1 $C3 > gpurun_out/r4j_w_$n.json 2> gpurun_out/r4j_w_$n.err || { echo "pmc $n failed"; exit 1; }
done
echo r4j done
