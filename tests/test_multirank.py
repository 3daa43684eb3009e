"""N > 1 path on CPU (gloo): row interleave + one gather + un-permute.

The per-rank renderer here is the oracle (CPU) on the rank's rows, standing in
for the GPU kernel; the sharding code is the one bench.py runs over RCCL
(nrt/shard.py).  The reassembled frame must equal the single-process render
bit for bit (RNG keyed by pixel index).
"""
import os
import socket
import tempfile

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from helpers import oracle_render, oracle_tree
from nrt import shard

SCENE, W, SPP = "scenes/cornell-box-scene.json", 12, 2


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, tree, out_path, H):
    os.environ["HSA_ENABLE_IPC_MODE_LEGACY"] = "0"
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=rank, world_size=world)
    try:
        rows = shard.rows_of(H, rank, world)
        img, _ = oracle_render(tree, rows=(rank, world), threads=1)
        buf = torch.zeros((shard.rows_max(H, world), W, 3), dtype=torch.float32)
        buf[:rows] = torch.from_numpy(img.reshape(rows, W, 3))
        frame = shard.gather_frame(buf, H, dist, rank, world)
        into = torch.full((H, W, 3), -1.0) if rank == 0 else None  # bench.py's path: un-permute into `out`
        for _ in range(2):  # (the second step reuses the cached staging tensor)
            framed = shard.gather_frame(buf, H, dist, rank, world, out=into)
        if rank == 0:
            assert framed is into
            np.save(out_path, np.stack([frame.numpy(), into.numpy()]))
        dist.barrier()
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
@pytest.mark.parametrize("H", [13, 12])  # ragged last shard / equal shards
def test_row_sharded_gather_matches_single_render(world, H):
    with tempfile.TemporaryDirectory() as td:
        tree, _ = oracle_tree(SCENE, td, width=W, height=H, spp=SPP)
        want, _ = oracle_render(tree, threads=2)
        out = os.path.join(td, "frame.npy")
        mp.spawn(_worker, args=(world, _free_port(), tree, out, H), nprocs=world, join=True)
        got = np.load(out)
    assert got.shape == (2, H, W, 3)
    np.testing.assert_array_equal(got[0].reshape(-1), want)
    np.testing.assert_array_equal(got[1].reshape(-1), want)


def test_shard_bookkeeping():
    for h in (1, 2, 7, 13, 1024):
        for n in (1, 2, 3, 8):
            assert sum(shard.rows_of(h, r, n) for r in range(n)) == h
            assert max(shard.rows_of(h, r, n) for r in range(n)) == shard.rows_max(h, n)
    parts = [torch.arange(r, 14, 3, dtype=torch.float32).repeat_interleave(3).reshape(-1, 1, 3) for r in range(3)]
    rmax = max(p.shape[0] for p in parts)
    padded = [torch.cat([p, torch.full((rmax - p.shape[0], 1, 3), -1.0)]) for p in parts]
    frame = shard.assemble(padded, 14)
    assert frame[:, 0, 0].tolist() == list(range(14))
