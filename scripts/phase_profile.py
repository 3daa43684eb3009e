"""Diagnostic: per-phase cycle shares of the render loop (s_memtime stamps).

usage: python scripts/phase_profile.py [scene] [variant ...]   variant = precision/rng/trace
"""
import json, os, sys
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nr-ray-tracer_amd"))
import nrt
os.chdir(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden"))
scene = sys.argv[1] if len(sys.argv) > 1 else "scenes/cornell-box-scene.json"
variants = sys.argv[2:] or ["f32/philox/auto", "f32/chacha8/auto", "f64/chacha8/auto"]
s = nrt.Scene.load(scene, nrt.CameraConfig(width=1024, height=1024, samples_per_pixel=32))
out = {}
for v in variants:
    prec, rng, trace = v.split("/")
    out[v] = s.phase_profile(precision=prec, rng=rng, trace=trace)
print(json.dumps(out, indent=1))
