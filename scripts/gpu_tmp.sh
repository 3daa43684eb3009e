set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread -k "f64 or exact or golden or kat or limits" > gpurun_out/gputest_pf.log 2>&1; rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/gputest_pf.log; [ $rc = 0 ] || exit 1
run() { # tag pf args
  local tag=$1 pf=$2; shift 2
  NRT_EXACT_PF=$pf timeout -k 10 200 python bench.py --no-cpu-baseline "$@" > gpurun_out/cfg_$tag.json 2>/dev/null || { echo "fail $tag"; return 1; }
  python -c "import json; d=json.load(open('gpurun_out/cfg_$tag.json')); print('$tag pf=$pf', d['value'], d['timings_ms']['kernel_device_only'], d['frame_sha256'][:16])"
}
for pf in 1 2; do
run c5f64 $pf --precision f64 --rng chacha8 --steps 1 --warmup 1 || exit 1
run c2f64 $pf --scene scenes/cornell-box-scene.json --width 512 --height 512 --spp 64 --precision f64 --rng chacha8 --steps 2 --warmup 1 || exit 1
done
run c4f64 1 --scene scenes/utah-teapot-scene.json --precision f64 --rng chacha8 --steps 1 --warmup 1 || exit 1
