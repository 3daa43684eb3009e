# Round-5 headline profile: C5 f32 Philox, pipelined default bench (kernel trace + PMC passes), and
# the same trace with --pipeline 0.
set -o pipefail
tag=${1:-r05}
bash scripts/profile.sh ${tag}_c5_f32_philox --steps 20 --warmup 2 || exit 1
python3 scripts/trace_period.py gpurun_out/prof_${tag}_c5_f32_philox/trace --json gpurun_out/prof_${tag}_c5_f32_philox/trace_period.json
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
mkdir -p gpurun_out/prof_${tag}_c5_p0 && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_${tag}_c5_p0/trace -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 20 --warmup 2 --pipeline 0 > gpurun_out/prof_${tag}_c5_p0/bench_trace.json 2> gpurun_out/prof_${tag}_c5_p0.err || exit 1
python3 scripts/trace_period.py gpurun_out/prof_${tag}_c5_p0/trace --json gpurun_out/prof_${tag}_c5_p0/trace_period.json
