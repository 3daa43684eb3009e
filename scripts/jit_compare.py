"""Diagnostic: the C5 frame from the scene-specialised (jit.hip) and the generic world-list
kernel, differing values and magnitude.  usage: python scripts/jit_compare.py"""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nr-ray-tracer_amd"))
import nrt
os.chdir(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden"))
s = nrt.Scene.load("scenes/cornell-box-scene.json", nrt.CameraConfig(width=1024, height=1024, samples_per_pixel=256))
os.environ["NRT_JIT"] = "0"
a = s.render(precision="f32", rng="philox")
os.environ["NRT_JIT"] = "1"
b = s.render(precision="f32", rng="philox")
print(nrt.LIB_PATH, nrt.jit_stats())
diff = a.view(np.uint32) != b.view(np.uint32)
px = diff.any(axis=2)
rel = np.abs(a - b).max(axis=2) / np.maximum(np.abs(a).max(axis=2), 1e-12)
print(f"values differing {diff.mean():.3e} pixels {px.sum()} of {px.size}, max rel {rel.max():.3e}, "
      f"channel means {a.reshape(-1,3).mean(0)} vs {b.reshape(-1,3).mean(0)}")
