# scratch GPU script (varies per experiment)
set -o pipefail
mkdir -p gpurun_out
bash scripts/configs_bench.sh pool5
