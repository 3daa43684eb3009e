# Every BASELINE config benched (scripts/configs_bench.sh), then the f32 profiles other than C5 re-taken
# (C4, C3, C2, C1, C1 at 1080p).  usage: bash scripts/gpu_configs_final.sh <tag>
#   then: python scripts/publish_profiles.py <tag> --as r06
set -o pipefail
tag=${1:-r6y}
mkdir -p gpurun_out
cd /tmp && export TMPDIR=/tmp && cd - >/dev/null
bash scripts/configs_bench.sh ${tag}_cfg > gpurun_out/${tag}_configs.log 2>&1 || { tail -5 gpurun_out/${tag}_configs.log; exit 1; }
cat gpurun_out/${tag}_configs.log
bash scripts/profile.sh ${tag}_c4_f32_philox --scene scenes/utah-teapot-scene.json --steps 8 --warmup 2 > gpurun_out/${tag}_p4.log 2>&1 || { tail -5 gpurun_out/${tag}_p4.log; exit 1; }
bash scripts/profile.sh ${tag}_c3_f32_philox --scene scenes/earth.toml --width 1920 --height 1080 --spp 128 --steps 3 --warmup 1 > gpurun_out/${tag}_p3.log 2>&1 || { tail -5 gpurun_out/${tag}_p3.log; exit 1; }
bash scripts/round_profile.sh ${tag} f32b > gpurun_out/${tag}_pb.log 2>&1 || { tail -5 gpurun_out/${tag}_pb.log; exit 1; }
echo profiles done
