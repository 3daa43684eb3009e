# Round-5 check of the library multi-GPU path, the JIT disk cache and the bench paths.
# usage: bash scripts/gpu_r5a.sh <tag>
set -o pipefail
tag=${1:-r5a}
mkdir -p gpurun_out
export NRT_JIT_CACHE=$PWD/gpurun_out/${tag}_jitcache
timeout -k 10 400 python -u -m pytest tests/test_multigpu.py tests/test_jit_cache.py tests/test_library.py tests/test_cli.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -40 gpurun_out/${tag}_pytest.log; exit 1; }
tail -3 gpurun_out/${tag}_pytest.log
for run in 1 2; do
  timeout -k 10 200 python bench.py --no-cpu-baseline > gpurun_out/${tag}_bench_default_$run.json 2> gpurun_out/${tag}_bench_default_$run.err || { tail -5 gpurun_out/${tag}_bench_default_$run.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('default', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['timings_s'], d['jit'], d['frame_sha256'][:16])" gpurun_out/${tag}_bench_default_$run.json
done
timeout -k 10 200 python bench.py --no-cpu-baseline --multi library --gpus 1 > gpurun_out/${tag}_bench_lib1.json 2> gpurun_out/${tag}_bench_lib1.err || { tail -5 gpurun_out/${tag}_bench_lib1.err; exit 1; }
python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print('lib1', d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d['multi_gpu'], d['timings_s'], d['frame_sha256'][:16])" gpurun_out/${tag}_bench_lib1.json
cd tests/golden
for run in 1 2; do
  /usr/bin/time -f "cli wall %e s" timeout -k 10 120 ../../nr-ray-tracer_amd/nrt/nrt-cli render scenes/cornell-box-scene.json -W 1024 -H 1024 --samples-per-pixel 256 --precision f32 --rng philox -v -f -o /tmp/c5.png 2>&1 | tail -3
done
