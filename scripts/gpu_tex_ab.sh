set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
C3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 128"
NRT_TEX_RGB8=1 timeout -k 10 300 python -u -m pytest tests/test_stat_parity.py tests/test_gpu_parity.py -m gpu -q -k "earth" --timeout 120 --timeout-method thread > gpurun_out/s12_pytest.log 2>&1; tail -2 gpurun_out/s12_pytest.log
timeout -k 10 300 python scripts/ab_configs.py --reps 3 --out gpurun_out/s12_ab.jsonl --env base="" --env rgb8="NRT_TEX_RGB8=1" --cfg c3="$C3" > gpurun_out/s12_ab.log 2>&1; tail -3 gpurun_out/s12_ab.log
for e in 0 1; do
  NRT_TEX_RGB8=$e timeout -s KILL 90 rocprofv3 --pmc FETCH_SIZE -d gpurun_out/s12_pmc_$e -o run --output-format csv -- python3 bench.py --no-cpu-baseline --kernel-only --steps 2 --warmup 1 $C3 > /dev/null 2> gpurun_out/s12_pmc_$e.err || { echo "pmc $e failed"; tail -3 gpurun_out/s12_pmc_$e.err; exit 1; }
  python3 scripts/pmc_summary.py gpurun_out/s12_pmc_$e --json gpurun_out/s12_pmc_$e.json > /dev/null
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('rgb8', sys.argv[2], 'FETCH_SIZE KiB/dispatch', d['per_dispatch'].get('FETCH_SIZE'))" gpurun_out/s12_pmc_$e.json $e
done
timeout -k 10 400 python scripts/ab_configs.py --reps 2 --out gpurun_out/s12_ab2.jsonl --lib cur=nr-ray-tracer_amd/nrt/libnrt.so --lib ifif=nr-ray-tracer_amd/ab/ifif/libnrt.so --env base="" --env ww24="NRT_WAVE_WAIT=24" --cfg c1="--scene scenes/spheres.toml --width 1920 --height 1080 --spp 64" > gpurun_out/s12_ab2.log 2>&1; tail -5 gpurun_out/s12_ab2.log
