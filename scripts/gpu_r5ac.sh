# Phase profile of the persistent exact walk (C5, C4) with candidate lists of 2.
set -o pipefail
tag=${1:-r5ac}
mkdir -p gpurun_out
for sc in cornell-box-scene.json utah-teapot-scene.json; do
NRT_LIB=$PWD/nr-ray-tracer_amd/ab/prof/libnrt.so timeout -k 10 120 python scripts/phase_profile.py scenes/$sc f64/chacha8/auto > gpurun_out/${tag}_phase_$sc || exit 1
cat gpurun_out/${tag}_phase_$sc
done
