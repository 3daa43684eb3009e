"""Strong-scaling headroom of the render kernel on one GPU: kernel time of rank 0's
row shard (rows y = 0 mod N) for N = 1, 2, 4, 8, against 1/N of the full frame.

usage: python scripts/shard_timing.py [scene] [W H spp] [N,N,...]
SHARD_MAX_BOUNCES=B overrides the scene's bounce cap (diagnostic: how much of the fixed per-launch
loss is the longest paths' serial bounces).
Each N is timed two ways: `shard_ms` brackets one launch with events after a synchronize (the host's
launch work, occupancy queries and hipModuleLaunchKernel, counts when the GPU waits for it), and
`shard_ms_queued` the same launch enqueued behind a previous one, so the GPU is still busy while the
host prepares it (as in bench.py's double-buffered loop): the kernel alone.
"""
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "nr-ray-tracer_amd"))
import nrt  # noqa: E402

scene = sys.argv[1] if len(sys.argv) > 1 else "scenes/cornell-box-scene.json"
W, H, spp = (int(v) for v in sys.argv[2:5]) if len(sys.argv) > 4 else (1024, 1024, 256)
os.chdir(os.path.join(ROOT, "tests", "golden"))
mb = int(os.environ["SHARD_MAX_BOUNCES"]) if os.environ.get("SHARD_MAX_BOUNCES") else None
s = nrt.Scene.load(scene, nrt.CameraConfig(width=W, height=H, samples_per_pixel=spp, ray_max_bounces=mb))
s.upload(0)
buf = torch.zeros((H, W, 3), dtype=torch.float32, device="cuda:0")
stream = torch.cuda.current_stream()
res, resq = {}, {}
ns = [int(v) for v in sys.argv[5].split(",")] if len(sys.argv) > 5 else [1, 2, 4, 8]
for n in ns:
    rows = (H + n - 1) // n
    launch = lambda: s.render_device(buf.data_ptr(), rows * W * 3, row_offset=0, row_stride=n,
                                     stream=stream.cuda_stream)
    times, queued = [], []
    for it in range(4):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        launch()
        e1.record(stream)
        torch.cuda.synchronize()
        if it:
            times.append(e0.elapsed_time(e1))
        launch()  # (still running while the timed launch below is prepared and enqueued)
        q0, q1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        q0.record(stream)
        launch()
        q1.record(stream)
        torch.cuda.synchronize()
        if it:
            queued.append(q0.elapsed_time(q1))
    res[n] = sum(times) / len(times)
    resq[n] = sum(queued) / len(queued)
base, baseq = res[ns[0]] * ns[0], resq[ns[0]] * ns[0]
out = {f"N={n}": {"shard_ms": round(t, 3), "efficiency_vs_N1": round(base / (n * t), 4),
                  "shard_ms_queued": round(resq[n], 3), "efficiency_queued": round(baseq / (n * resq[n]), 4)}
       for n, t in res.items()}
out["env"] = {k: v for k, v in os.environ.items() if k.startswith(("NRT_", "SHARD_"))}
print(json.dumps(out))
