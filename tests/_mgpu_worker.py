"""Worker for tests/test_multigpu.py, started by torch.distributed.run (one process per rank).

Each rank renders the image rows y = rank (mod N) into a device buffer through
libnrt.so's C ABI (nrt_render_device), then the frame is assembled on rank 0 by
the same code bench.py runs (nrt/shard.gather_frame):
  --backend nccl : one GPU per rank, RCCL gather of the device buffers
  --backend gloo : every rank on cuda:0, the device buffers copied to the host and
                   gathered over gloo (a one-GPU box still runs the shard renders of
                   several processes on the hardware)
Rank 0 writes the frames (one per precision/RNG variant) to --out as .npy.
"""
import argparse
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, os.path.join(ROOT, "nr-ray-tracer_amd"))
sys.path.insert(0, HERE)

import nrt  # noqa: E402
from nrt import shard  # noqa: E402
from helpers import in_golden  # noqa: E402

VARIANTS = [("f32", "philox"), ("f64", "chacha8")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--backend", choices=["nccl", "gloo"], required=True)
    ap.add_argument("--scene", default="scenes/cornell-box-scene.json")
    ap.add_argument("--width", type=int, default=64)
    ap.add_argument("--height", type=int, default=37)
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--out", required=True)
    a = ap.parse_args()
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    local = int(os.environ.get("LOCAL_RANK", "0")) if a.backend == "nccl" else 0
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    if a.backend == "nccl":
        dist.init_process_group("nccl", device_id=dev)
    else:
        dist.init_process_group("gloo")
    try:
        with in_golden():
            s = nrt.Scene.load(a.scene, nrt.CameraConfig(width=a.width, height=a.height, samples_per_pixel=a.spp))
        H, W = s.camera.height, s.camera.width
        rows = shard.rows_of(H, rank, world)
        frames = []
        for precision, rng in VARIANTS:
            buf = torch.zeros((shard.rows_max(H, world), W, 3), dtype=torch.float32, device=dev)
            s.render_device(buf.data_ptr(), rows * W * 3, precision=precision, rng=rng, device=local,
                            row_offset=rank, row_stride=world, stream=torch.cuda.current_stream().cuda_stream)
            torch.cuda.synchronize()
            if a.backend == "nccl":
                out = torch.empty((H, W, 3), dtype=torch.float32, device=dev) if rank == 0 else None
                frame = shard.gather_frame(buf, H, dist, rank, world, out=out)
            else:
                frame = shard.gather_frame(buf.cpu(), H, dist, rank, world)
            if rank == 0:
                frames.append(frame.cpu().numpy())
        if rank == 0:
            np.save(a.out, np.stack(frames))
        dist.barrier()
    finally:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
