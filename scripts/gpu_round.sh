# End-of-round evidence run: GPU tests, round profile (trace + PMC + default bench line),
# every single-GPU BASELINE config, phase profiles.  usage: bash scripts/gpu_round.sh <tag>
set -o pipefail
tag=${1:-r01}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${tag}_pytest.log 2>&1 || { tail -30 gpurun_out/${tag}_pytest.log; exit 1; }
tail -1 gpurun_out/${tag}_pytest.log
for part in f32a f32b f64; do
  bash scripts/round_profile.sh ${tag} $part > gpurun_out/${tag}_round_profile_$part.log 2>&1 || { tail -5 gpurun_out/${tag}_round_profile_$part.log; exit 1; }
  tail -1 gpurun_out/${tag}_round_profile_$part.log
done
bash scripts/configs_bench.sh ${tag}_cfg || exit 1
timeout -k 10 200 python scripts/phase_profile.py scenes/cornell-box-scene.json f32/philox/auto f32/chacha8/auto > gpurun_out/${tag}_phase.json 2>/dev/null || exit 1
timeout -k 10 200 python scripts/shard_timing.py > gpurun_out/${tag}_shard_c5.json 2>/dev/null || exit 1
timeout -k 10 300 python bench.py > gpurun_out/${tag}_bench_default.json 2> gpurun_out/${tag}_bench_default.err || exit 1
echo done
