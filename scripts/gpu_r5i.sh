# Three frames in flight: multi-GPU tests, default bench lines (D = 3, 2, 1), library path, shard timing.
set -o pipefail
tag=${1:-r5i}
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_multigpu.py tests/test_library.py -m gpu -x -q --timeout 150 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -2 gpurun_out/${tag}_pytest.log
show() { python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read())
print(sys.argv[2], d['value'], d['ms_per_step'], d['roofline']['kernel_ms'], d.get('pipeline',{}).get('frames_in_flight'), d['frame_sha256'][:16])" $1 $2; }
for rep in 1 2; do
  for p in 3 2 1; do
    f=gpurun_out/${tag}_p${p}_$rep
    timeout -k 10 200 python bench.py --no-cpu-baseline --pipeline $p > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
    show $f.json "pipeline=$p" || exit 1
  done
done
f=gpurun_out/${tag}_lib1
timeout -k 10 200 python bench.py --no-cpu-baseline --multi library --gpus 1 > $f.json 2> $f.err || { tail -5 $f.err; exit 1; }
show $f.json lib1
timeout -k 10 240 python scripts/shard_timing.py > gpurun_out/${tag}_shard.json 2>gpurun_out/${tag}_shard.err && cat gpurun_out/${tag}_shard.json
