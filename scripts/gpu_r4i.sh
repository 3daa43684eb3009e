set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r4i_pytest.log 2>&1 || { tail -30 gpurun_out/r4i_pytest.log; exit 1; }
tail -1 gpurun_out/r4i_pytest.log
timeout -k 10 150 python scripts/shard_timing.py > gpurun_out/r4i_shard.json && cat gpurun_out/r4i_shard.json || exit 1
timeout -k 10 200 python bench.py > gpurun_out/r4i_bench.json 2> gpurun_out/r4i_bench.err || { tail -5 gpurun_out/r4i_bench.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4i_bench.json')); print('bench', d['value'], d['timings_ms'], d['kernel_variant'], d['roofline']['frac'])"
timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 2 --backend gloo --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/r4i_bench_n2gloo.json 2> gpurun_out/r4i_bench_n2gloo.err || { tail -5 gpurun_out/r4i_bench_n2gloo.err; exit 1; }
python3 -c "import json; d=json.load(open('gpurun_out/r4i_bench_n2gloo.json')); e=json.load(open('gpurun_out/r4i_bench.json')); print('n2 gloo sha equal:', d['frame_sha256']==e['frame_sha256'], d['kernel_variant'])"
