"""Diagnostic: per-phase cycle shares of the render loop (s_memtime stamps)."""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nr-ray-tracer_amd"))
import nrt
os.chdir(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden"))
scene = sys.argv[1] if len(sys.argv) > 1 else "scenes/cornell-box-scene.json"
s = nrt.Scene.load(scene, nrt.CameraConfig(width=1024, height=1024, samples_per_pixel=32))
out = {}
for prec, rng in (("f32", "philox"), ("f32", "chacha8"), ("f64", "chacha8")):
    out[f"{prec}_{rng}"] = s.phase_profile(precision=prec, rng=rng)
print(json.dumps(out, indent=1))
