# scratch GPU script (varies per experiment): VALU cost microbench, bench A/B of library variants, round profile
set -o pipefail
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 120 scripts/ubench/valu_cost > gpurun_out/ubench_valu.jsonl 2>&1 && cat gpurun_out/ubench_valu.jsonl || { echo "ubench failed"; exit 1; }
for v in default nr-ray-tracer_amd/build/w7/libnrt.so nr-ray-tracer_amd/build/w8/libnrt.so; do
  tag=$(basename $(dirname $v))
  if [ $v != default ]; then export NRT_LIB=$PWD/$v; else unset NRT_LIB; fi
  timeout -k 10 120 python bench.py --no-cpu-baseline > gpurun_out/t_$tag.json 2>gpurun_out/t_$tag.err || { tail -3 gpurun_out/t_$tag.err; exit 1; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Msamples/s', d['roofline']['kernel_ms'], 'ms')" gpurun_out/t_$tag.json $tag
done
unset NRT_LIB
bash scripts/round_profile.sh r01d
