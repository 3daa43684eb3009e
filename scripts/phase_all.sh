# Phase profiles (PROF build of the f32 Philox loop, s_memtime stamps) of C4, C3 and C5 at spp 16:
# the source of profiles/r04_phase_profile.json.  usage: bash scripts/phase_all.sh [out.json]
set -o pipefail
mkdir -p gpurun_out
out=${1:-gpurun_out/phase_all.json}
timeout -k 10 300 python - <<'PY' > $out
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
