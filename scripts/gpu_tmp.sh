# scratch GPU script (varies per experiment): GPU tests, bench A/B of library variants
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/t_pytest.log 2>&1 || { tail -30 gpurun_out/t_pytest.log; exit 1; }
tail -2 gpurun_out/t_pytest.log
for v in default $VARIANTS default; do
  tag=$(basename $(dirname $v))
  if [ $v != default ]; then export NRT_LIB=$PWD/$v; else unset NRT_LIB; tag=default; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/t_$tag.json 2>gpurun_out/t_$tag.err || { tail -3 gpurun_out/t_$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Msamples/s', d['roofline']['kernel_ms'], 'ms')" gpurun_out/t_$tag.json $tag
done
if [ -n "$PROF" ]; then
  timeout -k 10 120 rocprofv3 --kernel-trace --stats -d gpurun_out/tprof -o run --output-format csv -- python3 bench.py --no-cpu-baseline --steps 2 > /dev/null 2>&1 && head -3 gpurun_out/tprof/run_kernel_stats.csv
fi
