"""Strong-scaling headroom of the render kernel on one GPU: kernel time of rank 0's
row shard (rows y = 0 mod N) for N = 1, 2, 4, 8, against 1/N of the full frame.

usage: python scripts/shard_timing.py [scene] [W H spp] [N,N,...]
SHARD_MAX_BOUNCES=B overrides the scene's bounce cap (diagnostic: how much of the fixed per-launch
loss is the longest paths' serial bounces).
Each N is timed two ways: `shard_ms` brackets one launch with events after a synchronize (the host's
launch work, occupancy queries and hipModuleLaunchKernel, counts when the GPU waits for it), and
`shard_ms_queued` the same launch enqueued behind a previous one, so the GPU is still busy while the
host prepares it (as in bench.py's double-buffered loop): the kernel alone.  `shard_ms_pipelined`:
K launches alternating over SHARD_STREAMS (default 2, as bench.py and the library) streams and buffers (the library's multi-GPU render does this,
csrc/multi.hip), total device time / K: launch k+1's workgroups take the SIMDs launch k's last paths
leave idle, so the per-launch tail overlaps the next launch's start.
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
NSTREAMS = int(os.environ.get("SHARD_STREAMS", "2"))  # pipelined mode: launches in flight
pbufs = [buf] + [torch.zeros_like(buf) for _ in range(NSTREAMS - 1)]
pstreams = [stream] + [torch.cuda.Stream(device="cuda:0") for _ in range(NSTREAMS - 1)]
res, resq, resp = {}, {}, {}
K = int(os.environ.get("SHARD_K", "8"))  # launches per pipelined measurement (the last one's tail is not overlapped)
ns = [int(v) for v in sys.argv[5].split(",")] if len(sys.argv) > 5 else [1, 2, 4, 8]
# one-shot launches (shard_ms, shard_ms_queued) group their pixels as nrt_render does (16 Philox groups per
# resident wave, api.cpp ONE_SHOT_GROUPS_PER_WAVE), pipelined ones as nrt_render_device does (4): the env knob
# stands in for the API's choice here, unless the caller fixed it
GPW_FIXED = os.environ.get("NRT_GROUPS_PER_WAVE")
for n in ns:
    rows = (H + n - 1) // n
    launch = lambda: s.render_device(buf.data_ptr(), rows * W * 3, row_offset=0, row_stride=n,
                                     stream=stream.cuda_stream)
    if not GPW_FIXED:
        os.environ["NRT_GROUPS_PER_WAVE"] = "16"
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
    piped = []
    if not GPW_FIXED:
        os.environ.pop("NRT_GROUPS_PER_WAVE", None)
    for it in range(3):
        torch.cuda.synchronize()
        p0, p1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        p0.record(stream)
        for st in pstreams[1:]:
            st.wait_event(p0)
        for k in range(K):
            st, b = pstreams[k % NSTREAMS], pbufs[k % NSTREAMS]
            s.render_device(b.data_ptr(), rows * W * 3, row_offset=0, row_stride=n, stream=st.cuda_stream)
        for st in pstreams[1:]:
            done = torch.cuda.Event()
            done.record(st)
            stream.wait_event(done)
        p1.record(stream)
        torch.cuda.synchronize()
        piped.append(p0.elapsed_time(p1) / K)
    resp[n] = min(piped)
base, baseq, basep = res[ns[0]] * ns[0], resq[ns[0]] * ns[0], resp[ns[0]] * ns[0]
out = {f"N={n}": {"shard_ms": round(t, 3), "efficiency_vs_N1": round(base / (n * t), 4),
                  "shard_ms_queued": round(resq[n], 3), "efficiency_queued": round(baseq / (n * resq[n]), 4),
                  "shard_ms_pipelined": round(resp[n], 3), "efficiency_pipelined": round(basep / (n * resp[n]), 4),
                  "efficiency_pipelined_vs_unpipelined_N1": round(base / (n * resp[n]), 4)}
       for n, t in res.items()}
out["env"] = {k: v for k, v in os.environ.items() if k.startswith(("NRT_", "SHARD_"))}
out["groups_per_wave"] = {"one_shot": GPW_FIXED or "16 (nrt_render)", "pipelined": GPW_FIXED or "4 (nrt_render_device)"}
print(json.dumps(out))
