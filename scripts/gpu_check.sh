# GPU check: parity tests then a short bench of each kernel variant.
# usage: bash scripts/gpu_check.sh <tag>
set -o pipefail
tag=${1:-run}
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -m gpu -q > gpurun_out/${tag}_pytest_gpu.log 2>&1; echo "pytest rc=$?" >> gpurun_out/${tag}_pytest_gpu.log
tail -4 gpurun_out/${tag}_pytest_gpu.log
for v in "f32 chacha8 auto" "f32 philox auto" "f32 philox bvh" "f64 chacha8 auto" "f64 philox auto"; do set -- $v
  f=gpurun_out/${tag}_bench_$1_$2_$3
  timeout -k 10 240 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --precision $1 --rng $2 --trace $3 > $f.json 2> $f.err || { echo "bench $1 $2 $3 failed rc=$?"; tail -3 $f.err; break; }
  python3 -c "import json,sys; d=json.load(open(sys.argv[1])); print(sys.argv[2], d['value'], 'Msamples/s', d['roofline']['kernel_ms'], 'ms')" $f.json "$1/$2/$3"
done
