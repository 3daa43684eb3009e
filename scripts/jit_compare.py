"""The full C5 frame (or another scene's) from the scene-specialised (jit.hip) and the generic
kernel: sha256 of both, differing values and magnitude.  They must be equal bit for bit
(kernel.hpp fmad: both builds contract with -ffp-contract=on).
usage: python scripts/jit_compare.py [scene W H spp [trace]]"""
import hashlib
import os
import sys

import numpy as np

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nr-ray-tracer_amd"))
import nrt

a = sys.argv[1:]
scene = a[0] if a else "scenes/cornell-box-scene.json"
w, h, spp = (int(x) for x in a[1:4]) if len(a) >= 4 else (1024, 1024, 256)
trace = a[4] if len(a) >= 5 else "auto"
os.chdir(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden"))
s = nrt.Scene.load(scene, nrt.CameraConfig(width=w, height=h, samples_per_pixel=spp))
os.environ["NRT_JIT"] = "0"
g = s.render(precision="f32", rng="philox", trace=trace)
os.environ["NRT_JIT"] = "1"
j = s.render(precision="f32", rng="philox", trace=trace)
diff = g.view(np.uint32) != j.view(np.uint32)
px = diff.any(axis=2)
rel = np.abs(g - j).max(axis=2) / np.maximum(np.abs(g).max(axis=2), 1e-12)
print(f"{scene} {w}x{h} spp={spp} trace={trace} jit={nrt.jit_stats()}")
print(f"sha256 generic {hashlib.sha256(g.tobytes()).hexdigest()}")
print(f"sha256 jit     {hashlib.sha256(j.tobytes()).hexdigest()}")
print(f"values differing {diff.mean():.3e}, pixels {px.sum()} of {px.size}, max rel {rel.max():.3e}")
sys.exit(1 if px.any() else 0)
