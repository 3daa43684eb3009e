set -o pipefail
mkdir -p gpurun_out
python - <<'PY' > gpurun_out/r4c_phase.json
import json, os, sys
sys.path.insert(0, "nr-ray-tracer_amd")
import nrt
os.chdir("tests/golden")
out = {}
for scene, w, h in (("scenes/utah-teapot-scene.json", 1024, 1024), ("scenes/earth.toml", 1920, 1080), ("scenes/cornell-box-scene.json", 1024, 1024)):
    s = nrt.Scene.load(scene, nrt.CameraConfig(width=w, height=h, samples_per_pixel=16))
    out[scene] = s.phase_profile(precision="f32", rng="philox", trace="auto")
print(json.dumps(out, indent=1))
PY
timeout -k 10 600 python scripts/ab_configs.py --reps 2 --out gpurun_out/r4c_ab.jsonl --lib A=nr-ray-tracer_amd/ab/on1/libnrt.so --lib B=nr-ray-tracer_amd/nrt/libnrt.so --cfg c3="--scene scenes/earth.toml --width 1920 --height 1080 --spp 128" --cfg c1big="--scene scenes/spheres.toml --width 1920 --height 1080 --spp 64" 2>&1 | tail -6
