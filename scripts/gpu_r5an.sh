# Spheres scene (C1) through the reference-exact kernel: speed and phase split.
set -o pipefail
tag=${1:-r5an}
mkdir -p gpurun_out
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --warmup 1 --scene scenes/spheres.toml --width 1920 --height 1080 --spp 64 --precision f64 --rng chacha8 > gpurun_out/${tag}_c1big_f64.json 2> gpurun_out/${tag}_c1big_f64.err || { tail -5 gpurun_out/${tag}_c1big_f64.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('c1big f64', d['value'], d['roofline']['kernel_ms'], d.get('kernel_variant'), d['roofline'].get('pmc',{}).get('kernel','')[:150])" gpurun_out/${tag}_c1big_f64.json
timeout -k 10 300 python bench.py --no-cpu-baseline --steps 4 --warmup 1 --scene scenes/spheres.toml --width 400 --height 225 --spp 16 --precision f64 --rng chacha8 > gpurun_out/${tag}_c1_f64.json 2> gpurun_out/${tag}_c1_f64.err || { tail -5 gpurun_out/${tag}_c1_f64.err; exit 1; }
python3 -c "
import json,sys
d=json.loads(open(sys.argv[1]).read().strip().splitlines()[-1])
print('c1 f64', d['value'], d['roofline']['kernel_ms'])" gpurun_out/${tag}_c1_f64.json
timeout -k 10 120 python scripts/phase_profile.py scenes/spheres.toml f64/chacha8/auto > gpurun_out/${tag}_phase_c1.json || exit 1
cat gpurun_out/${tag}_phase_c1.json
