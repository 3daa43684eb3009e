# A/B timing of two libnrt.so builds on the same box (alternating runs).
# usage: bash scripts/ab.sh <libA> <libB> [reps] [bench args...]
set -o pipefail
a=$1; b=$2; n=${3:-3}; shift 3
for i in $(seq 1 $n); do
  for lib in "$a" "$b"; do
    NRT_LIB=$PWD/$lib timeout -k 10 120 python bench.py --no-cpu-baseline "$@" > /tmp/ab_line.json || exit 1
    python -c "import json,sys; d=json.load(open('/tmp/ab_line.json')); print('$lib', d['value'], d['timings_ms']['kernel_device_only'])"
  done
done
