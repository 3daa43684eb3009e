"""Diagnostic: localise a statistical bias between two f32 traversal modes (world list vs instance BVH).
Renders the same frame at high spp for several bounce caps and stores both in an .npz under gpurun_out/."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nr-ray-tracer_amd"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import nrt  # noqa: E402
from helpers import in_golden  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "scenes/cornell-box-scene.json"
w = h = int(sys.argv[2]) if len(sys.argv) > 2 else 64
spp = int(sys.argv[3]) if len(sys.argv) > 3 else 65536
out = {}
for b in (1, 2, 3, 4, 50):
    with in_golden():
        s = nrt.Scene.load(scene, nrt.CameraConfig(width=w, height=h, samples_per_pixel=spp, ray_max_bounces=b))
    for mode in ("auto", "bvh", "world-bvh"):
        img = s.render(precision="f32", rng="philox", trace=mode)
        out[f"{mode}_{b}"] = img
        print(b, mode, img.reshape(-1, 3).mean(0), flush=True)
    img = s.render(precision="f64", rng="philox")
    out[f"f64_{b}"] = img
    print(b, "f64", img.reshape(-1, 3).mean(0), flush=True)
os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
np.savez_compressed(os.path.join(ROOT, "gpurun_out", "debug_bias.npz"), **out)
