import json, os, sys
sys.path.insert(0, "nr-ray-tracer_amd")
import nrt
os.chdir("tests/golden")
out = {}
for spp in (16, 256):
    s = nrt.Scene.load("scenes/utah-teapot-scene.json", nrt.CameraConfig(width=1024, height=1024, samples_per_pixel=spp))
    out[spp] = s.phase_profile(precision="f32", rng="philox", trace="auto")
print(json.dumps(out, indent=1))
