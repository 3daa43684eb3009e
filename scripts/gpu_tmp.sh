set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/r1ww_pytest.log 2>&1; tail -3 gpurun_out/r1ww_pytest.log
for wv in 1 8 16 24 32 48; do
  NRT_WAVE_WAIT=$wv timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --scene scenes/utah-teapot-scene.json > gpurun_out/ww_$wv.json 2>gpurun_out/ww_$wv.err || { echo fail $wv; break; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('wait', sys.argv[2], d['value'])" gpurun_out/ww_$wv.json $wv
done
NRT_WAVE_WAIT=16 timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --scene scenes/spheres.toml --width 1920 --height 1080 --spp 64 > gpurun_out/ww_sph.json && python3 -c "import json; print('spheres', json.load(open('gpurun_out/ww_sph.json'))['value'])"
