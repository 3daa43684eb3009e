# Round-5 configs run (bench.py per BASELINE config and kernel variant), then the pipelined shard timing.
set -o pipefail
tag=${1:-r05cfg}
bash scripts/configs_bench.sh $tag || exit 1
timeout -k 10 240 python scripts/shard_timing.py > gpurun_out/${tag}_shard.json 2>gpurun_out/${tag}_shard.err && cat gpurun_out/${tag}_shard.json
