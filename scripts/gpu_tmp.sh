set -o pipefail
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/r02_bench_default.json 2> gpurun_out/r02_bench_default.err || { tail -5 gpurun_out/r02_bench_default.err; exit 1; }
cat gpurun_out/r02_bench_default.json | cut -c1-400
bash scripts/configs_bench.sh r02cfg
