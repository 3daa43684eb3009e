set -o pipefail
timeout -k 10 600 python -m pytest tests -m gpu -q > gpurun_out/r1b6_pytest.log 2>&1; tail -2 gpurun_out/r1b6_pytest.log
for var in default b; do
  lib=""; [ $var != default ] && lib=$PWD/nr-ray-tracer_amd/build/var_$var/libnrt.so
  for v in 1 0; do
    for sc in "scenes/utah-teapot-scene.json" "scenes/spheres.toml --width 1920 --height 1080 --spp 64"; do
      NRT_LIB=$lib NRT_WBVH4=$v timeout -k 10 200 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --scene $sc > gpurun_out/b4.json 2>gpurun_out/b4.err || { echo fail; tail -3 gpurun_out/b4.err; exit 1; }
      python3 -c "import json,sys; d=json.load(open('gpurun_out/b4.json')); print(sys.argv[1], 'wbvh4', sys.argv[2], d['config']['scene'], d['value'])" $var $v
    done
  done
done
