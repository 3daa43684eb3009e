# Round-5 profiles of every single-GPU config's default kernel and the reference-exact kernels
# (kernel trace + stats, PMC passes, trace period), one part per gpurun call.
# usage: bash scripts/gpu_r5prof.sh f32a|f32b|f64
set -o pipefail
part=${1:-f32a}
bash scripts/round_profile.sh r05 $part || exit 1
for d in gpurun_out/prof_r05_*; do
  [ -f $d/trace_period.json ] || python3 scripts/trace_period.py $d/trace --json $d/trace_period.json > /dev/null || true
done
echo "profiles $part done"
