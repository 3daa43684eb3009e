# Round-5 check of the library multi-GPU path, the JIT disk cache, frame pipelining and the bench paths.
# usage: bash scripts/gpu_r5a.sh <tag>
set -o pipefail
tag=${1:-r5a}
mkdir -p gpurun_out
export NRT_JIT_CACHE=$PWD/gpurun_out/${tag}_jitcache
timeout -k 10 400 python -u -m pytest tests/test_multigpu.py tests/test_jit_cache.py tests/test_library.py tests/test_cli.py -m gpu -x -v --timeout 150 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -40 gpurun_out/${tag}_pytest.log; exit 1; }
tail -3 gpurun_out/${tag}_pytest.log
show() { python3 -c "
import json,sys
l=[x for x in open(sys.argv[1]) if x.startswith('{')]
assert len(l)==1 and open(sys.argv[1]).read().startswith('{'), 'stdout is not one JSON line'
d=json.loads(l[0]); print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d.get('pipeline'), d.get('multi_gpu'), d['timings_s'], d['frame_sha256'][:16])" $1 $2; }
for run in 1 2; do
  for p in 1 0; do
    f=gpurun_out/${tag}_bench_p${p}_$run
    timeout -k 10 200 python bench.py --no-cpu-baseline --pipeline $p > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    show $f.json "pipeline=$p" || exit 1
  done
  f=gpurun_out/${tag}_bench_lib1_$run
  timeout -k 10 200 python bench.py --no-cpu-baseline --multi library --gpus 1 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
  show $f.json lib1 || exit 1
done
timeout -k 10 240 python scripts/shard_timing.py > gpurun_out/${tag}_shard.json 2>gpurun_out/${tag}_shard.err || { tail -5 gpurun_out/${tag}_shard.err; exit 1; }
cat gpurun_out/${tag}_shard.json
cd tests/golden
TIMEFORMAT="cli wall %R s"
for run in 1 2; do
  time timeout -k 10 120 ../../nr-ray-tracer_amd/nrt/nrt-cli render scenes/cornell-box-scene.json -W 1024 -H 1024 --samples-per-pixel 256 --precision f32 --rng philox -v -f -o /tmp/c5.png
done
