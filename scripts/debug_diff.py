"""Debug: compare f32 (fast) vs f64 (exact) renders on the same ChaCha8 stream."""
import os, sys
import numpy as np
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "nr-ray-tracer_amd"))
import nrt
os.chdir(os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden"))
scene = sys.argv[1] if len(sys.argv) > 1 else "scenes/cube-scene.json"
for bounces in (1, 2, 3):
    s = nrt.Scene.load(scene, nrt.CameraConfig(width=96, height=72, samples_per_pixel=1, ray_max_bounces=bounces))
    a = s.render(precision="f32", rng="chacha8")
    b = s.render(precision="f64", rng="chacha8")
    d = np.abs(a - b).max(axis=2) > 1e-3
    print(f"bounces={bounces}: mismatching pixels {d.sum()} / {d.size}; mean f32 {a.mean():.5f} f64 {b.mean():.5f}")
    np.save(f"/root/repo/gpurun_out/dbg_{bounces}_f32.npy", a)
    np.save(f"/root/repo/gpurun_out/dbg_{bounces}_f64.npy", b)
