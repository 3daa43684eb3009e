# Pipelined shard timing: 256- vs 64-thread workgroups and 2 vs 3 launches in flight, alternating.
set -o pipefail
tag=${1:-r5g}
show() { python3 -c "
import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], {k:(v['shard_ms_pipelined'], v['efficiency_pipelined'], v['shard_ms']) for k,v in d.items() if k.startswith('N=')})" $1 $2; }
for rep in 1 2; do
  timeout -k 10 240 python scripts/shard_timing.py scenes/cornell-box-scene.json 1024 1024 256 1,4,8 > gpurun_out/${tag}_b256_$rep.json 2>gpurun_out/${tag}_b256_$rep.err || exit 1
  show gpurun_out/${tag}_b256_$rep.json b256
  NRT_LIB=$PWD/nr-ray-tracer_amd/ab/b64/libnrt.so NRT_JIT_DEFS=-DNRT_BLOCK=64 timeout -k 10 240 python scripts/shard_timing.py scenes/cornell-box-scene.json 1024 1024 256 1,4,8 > gpurun_out/${tag}_b64_$rep.json 2>gpurun_out/${tag}_b64_$rep.err || exit 1
  show gpurun_out/${tag}_b64_$rep.json b64
  SHARD_STREAMS=3 timeout -k 10 240 python scripts/shard_timing.py scenes/cornell-box-scene.json 1024 1024 256 1,4,8 > gpurun_out/${tag}_s3_$rep.json 2>gpurun_out/${tag}_s3_$rep.err || exit 1
  show gpurun_out/${tag}_s3_$rep.json s3
done
