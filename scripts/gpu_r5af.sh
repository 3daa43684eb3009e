# Round-5 exact-kernel profiles (persistent walk, record carry, two candidates) and the configs bench.
set -o pipefail
tag=${1:-r5af}
bash scripts/gpu_r5prof.sh f64 || exit 1
bash scripts/configs_bench.sh $tag || exit 1
