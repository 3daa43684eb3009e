"""Multi-process rendering on the hardware: the frame assembled from
row shards rendered by separate processes must equal the single-process render
bit for bit, because the RNG is keyed by pixel index (camera.rs:318-320) and
Philox pixel sums are exact.

  * RCCL, one process per visible GPU (skipped with fewer than two GPUs);
  * gloo, two processes sharing cuda:0 (runs on any GPU box: the shard renders of
    several processes on the same card, the host-side gather bench.py's code uses).

The launcher (torch.distributed.run) is a child process: nothing here execs.
"""
import os
import socket
import subprocess
import sys
import tempfile

import numpy as np
import pytest

import nrt
from helpers import ROOT, in_golden

pytestmark = pytest.mark.gpu

WORKER = os.path.join(ROOT, "tests", "_mgpu_worker.py")
SCENE, W, H, SPP = "scenes/cornell-box-scene.json", 64, 37, 8
VARIANTS = [("f32", "philox"), ("f64", "chacha8")]


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _single():
    with in_golden():
        s = nrt.Scene.load(SCENE, nrt.CameraConfig(width=W, height=H, samples_per_pixel=SPP))
    return [s.render(precision=p, rng=r, device=0) for p, r in VARIANTS]


def _launch(n, backend):
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "frames.npy")
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr=127.0.0.1", f"--master-port={_port()}", WORKER, "--backend", backend,
               "--scene", SCENE, "--width", str(W), "--height", str(H), "--spp", str(SPP), "--out", out]
        env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
        r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
        assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
        return np.load(out)


def test_rccl_row_shards_bitwise_identical():
    n = nrt.device_count()
    if n < 2:
        pytest.skip(f"{n} GPU visible: the RCCL gather needs one process per GPU on >= 2 GPUs")
    got = _launch(min(n, 8), "nccl")
    for frame, want, (p, r) in zip(got, _single(), VARIANTS):
        np.testing.assert_array_equal(frame, want, err_msg=f"{p}/{r}")


def test_shared_gpu_processes_bitwise_identical():
    got = _launch(2, "gloo")
    for frame, want, (p, r) in zip(got, _single(), VARIANTS):
        np.testing.assert_array_equal(frame, want, err_msg=f"{p}/{r}")


def _bench(n, extra=()):
    """bench.py's own N-rank step (launched as the driver does, torch.distributed.run as a child
    process) at a small size: its JSON line."""
    import json
    args = ["--gpus", str(n), "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--width", "64", "--height", "37",
            "--spp", "8", *extra]
    bench = os.path.join(ROOT, "bench.py")
    if n == 1:
        cmd = [sys.executable, bench, *args]
    else:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
               "--master-addr=127.0.0.1", f"--master-port={_port()}", bench, *args]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0", OMP_NUM_THREADS="1")
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    return json.loads(lines[0])


@pytest.mark.parametrize("precision,rng", VARIANTS)
def test_bench_multirank_step_matches_single(precision, rng):
    """bench.py's N > 1 step (row shards, one gather to rank 0, un-permute, max-over-ranks timing)
    runs end to end with two ranks sharing cuda:0 over gloo (the host-side gather; the RCCL
    path is the same code with the collective on the device) and assembles the frame the
    single-rank run renders, bit for bit (camera.rs:318-320: the RNG is keyed by pixel)."""
    one = _bench(1, ("--precision", precision, "--rng", rng))
    two = _bench(2, ("--precision", precision, "--rng", rng, "--backend", "gloo"))
    assert one["n_gpus"] == 1 and two["n_gpus"] == 2
    assert two["value"] > 0 and two["ms_per_step"] > 0
    assert one["frame_sha256"] and two["frame_sha256"] == one["frame_sha256"]


def test_render_on_second_device_keeps_current_device():
    """The library renders on the scene's device whatever the caller's current device is,
    and leaves the caller's current device unchanged (device guard, render.hip)."""
    n = nrt.device_count()
    if n < 2:
        pytest.skip(f"{n} GPU visible: needs two devices")
    torch = pytest.importorskip("torch")
    with in_golden():
        s = nrt.Scene.load(SCENE, nrt.CameraConfig(width=24, height=16, samples_per_pixel=2))
    want = s.render(precision="f64", rng="chacha8", device=0)
    torch.cuda.set_device(0)
    t = torch.empty((16, 24, 3), dtype=torch.float32, device="cuda:1")
    s.render_device(t.data_ptr(), t.numel(), precision="f64", rng="chacha8", device=1, stream=0)
    torch.cuda.synchronize(1)
    assert torch.cuda.current_device() == 0
    np.testing.assert_array_equal(t.cpu().numpy(), want)
    got = s.render(precision="f64", rng="chacha8", device=1)
    assert torch.cuda.current_device() == 0
    np.testing.assert_array_equal(got, want)
