"""Multi-process rendering on the hardware: the frame assembled from
row shards rendered by separate processes must equal the single-process render
bit for bit, because the RNG is keyed by pixel index (camera.rs:318-320) and
Philox pixel sums are exact.

  * RCCL, one process per visible GPU (skipped with fewer than two GPUs);
  * gloo, two processes sharing cuda:0 (runs on any GPU box: the shard renders of
    several processes on the same card, the host-side gather bench.py's code uses);
  * the library's own multi-GPU render in one process (nrt_render_opts.gpus, csrc/multi.hip:
    ncclCommInitAll + one ncclGather per frame): at N = 1 on any box (a communicator of one has
    nothing to exchange: the gather is a device copy), through RCCL at N >= 2 where the devices
    exist, and at N = 2, 3, 8 on one GPU through the test-only loopback
    (NRT_MULTI_LOOPBACK=1: the N shards on GPU 0, each shard's ncclGather a device-to-device copy
    into the same staging slot; the row counts, short shards, buffer-set rotation, event chaining
    and un-permute are the N-GPU code).

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


def _bench(n, extra=(), launcher=True):
    """bench.py's own N-rank step (launched as the driver does, torch.distributed.run as a child
    process; launcher=False: `python bench.py --gpus N` as is) at a small size: its JSON line."""
    import json
    args = ["--gpus", str(n), "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--width", "64", "--height", "37",
            "--spp", "8", *extra]
    bench = os.path.join(ROOT, "bench.py")
    if n == 1 or not launcher:
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


def test_bench_without_launcher_starts_its_ranks():
    """`python bench.py --gpus 2 --backend gloo` with no launcher (as a driver might invoke it): bench.py
    starts torch.distributed.run as a child process and forwards its line; the frame equals N = 1."""
    one = _bench(1)
    two = _bench(2, ("--backend", "gloo"), launcher=False)
    assert two["n_gpus"] == 2 and two["multi_gpu"]["path"] == "ranks"
    assert one["frame_sha256"] and two["frame_sha256"] == one["frame_sha256"]


@pytest.mark.parametrize("precision,rng", VARIANTS)
def test_library_multi_gpu_n1(precision, rng):
    """nrt_render_opts.gpus = 1: the frame goes through the library's multi-GPU path (buffer sets, the
    shard's copy into the staging buffer, the row un-permute) and equals the single-device render bit
    for bit."""
    with in_golden():
        s = nrt.Scene.load(SCENE, nrt.CameraConfig(width=W, height=H, samples_per_pixel=SPP))
    want = s.render(precision=precision, rng=rng, device=0)
    got = s.render(precision=precision, rng=rng, device=0, gpus=1)
    np.testing.assert_array_equal(got, want)
    t = s.render_timings()
    assert len(t["kernel_ms"]) == 1 and t["kernel_ms"][0] > 0 and t["gather_ms"] >= 0 and t["period_ms"] == 0


def test_library_multi_gpu_device_api_pipelined():
    """nrt_render_device with gpus = 1 into device memory, several frames enqueued back to back (the
    two buffer sets alternate): every frame equals the single-device render."""
    torch = pytest.importorskip("torch")
    with in_golden():
        s = nrt.Scene.load(SCENE, nrt.CameraConfig(width=W, height=H, samples_per_pixel=SPP))
    want = s.render(precision="f32", rng="philox", device=0)
    outs = [torch.empty((H, W, 3), dtype=torch.float32, device="cuda:0") for _ in range(5)]  # > the 3 buffer sets
    st = torch.cuda.current_stream(0)
    for o in outs:
        s.render_device(o.data_ptr(), o.numel(), precision="f32", rng="philox", device=0, stream=st.cuda_stream, gpus=1)
    torch.cuda.synchronize(0)
    for o in outs:
        np.testing.assert_array_equal(o.cpu().numpy(), want)


def test_bench_library_path_n1_matches_single():
    """bench.py --multi library (one process, the library's multi-GPU path) renders the frame of the
    default single-device path."""
    one = _bench(1)
    lib1 = _bench(1, ("--multi", "library"))
    assert lib1["multi_gpu"]["path"] == "library" and lib1["n_gpus"] == 1
    assert one["frame_sha256"] and lib1["frame_sha256"] == one["frame_sha256"]


@pytest.mark.parametrize("precision,rng", VARIANTS)
def test_library_multi_gpu_bitwise_identical(precision, rng):
    """nrt_render_opts.gpus = N >= 2 (every visible GPU, up to 8): the gathered, un-permuted frame equals
    the one-GPU frame bit for bit, also for a height that leaves the last shards a row short."""
    n = nrt.device_count()
    if n < 2:
        pytest.skip(f"{n} GPU visible: the library's multi-GPU render needs >= 2 devices")
    with in_golden():
        s = nrt.Scene.load(SCENE, nrt.CameraConfig(width=W, height=H, samples_per_pixel=SPP))
    want = s.render(precision=precision, rng=rng, device=0)
    for g in sorted({2, min(n, 8)}):
        got = s.render(precision=precision, rng=rng, device=0, gpus=g)
        np.testing.assert_array_equal(got, want, err_msg=f"gpus={g}")
        assert len(s.render_timings()["kernel_ms"]) == g


def test_bench_library_multi_gpu_matches_single():
    n = nrt.device_count()
    if n < 2:
        pytest.skip(f"{n} GPU visible: needs >= 2 devices")
    one = _bench(1)
    many = _bench(min(n, 8), launcher=False)  # no launcher, nccl: the library path
    assert many["multi_gpu"]["path"] == "library"
    assert many["frame_sha256"] == one["frame_sha256"]


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


LOOPBACK_N = (2, 3, 8)


@pytest.mark.parametrize("precision,rng", VARIANTS)
def test_library_multi_gpu_loopback_bitwise_identical(monkeypatch, precision, rng):
    """The library's N-GPU render (multi.hip) at N = 2, 3, 8 on one GPU (loopback): H = 37 leaves the last
    shards a row short at every N, and a 5-row frame leaves shards 5..7 of N = 8 empty; every frame equals
    the single-device render bit for bit (camera.rs:318-320: a pixel's value is a function of its index)."""
    monkeypatch.setenv("NRT_MULTI_LOOPBACK", "1")
    for h in (H, 5):
        with in_golden():
            s = nrt.Scene.load(SCENE, nrt.CameraConfig(width=W, height=h, samples_per_pixel=SPP))
        want = s.render(precision=precision, rng=rng, device=0)
        for g in LOOPBACK_N:
            got = s.render(precision=precision, rng=rng, device=0, gpus=g)
            np.testing.assert_array_equal(got, want, err_msg=f"gpus={g} H={h}")
            t = s.render_timings()
            assert len(t["kernel_ms"]) == g and t["gather_ms"] > 0


def test_library_multi_gpu_loopback_device_api_pipelined(monkeypatch):
    """nrt_render_device with gpus = 3 (loopback), seven frames enqueued back to back, alternating between
    two caller streams (GPU 0's gathers run on the caller's stream, chained to the previous frame's gather
    when it changes), then a different frame size (the shard buffers are re-made): every frame equals the
    single-device render."""
    torch = pytest.importorskip("torch")
    monkeypatch.setenv("NRT_MULTI_LOOPBACK", "1")
    with in_golden():
        s = nrt.Scene.load(SCENE, nrt.CameraConfig(width=W, height=H, samples_per_pixel=SPP))
    want = s.render(precision="f32", rng="philox", device=0)
    s.prepare(precision="f32", rng="philox", device=0, gpus=3)
    streams = [torch.cuda.Stream(device=0), torch.cuda.current_stream(0)]
    outs = [torch.full((H, W, 3), -1.0, dtype=torch.float32, device="cuda:0") for _ in range(7)]
    for k, o in enumerate(outs):
        s.render_device(o.data_ptr(), o.numel(), precision="f32", rng="philox", device=0,
                        stream=streams[k % 2].cuda_stream, gpus=3)
    torch.cuda.synchronize(0)
    for k, o in enumerate(outs):
        np.testing.assert_array_equal(o.cpu().numpy(), want, err_msg=f"frame {k}")
    t = s.render_timings()
    assert len(t["kernel_ms"]) == 3 and t["period_ms"] > 0
    import dataclasses
    small = dataclasses.replace(s.camera, height=16)
    o = torch.empty((16, W, 3), dtype=torch.float32, device="cuda:0")
    s.render_device(o.data_ptr(), o.numel(), camera=small, precision="f32", rng="philox", device=0,
                    stream=streams[0].cuda_stream, gpus=3)
    torch.cuda.synchronize(0)
    np.testing.assert_array_equal(o.cpu().numpy(), s.render(small, precision="f32", rng="philox", device=0))


def test_library_multi_gpu_prepare_and_stream_checks(monkeypatch):
    """nrt_render_prepare builds the N-GPU context before the first render (N = 1, loopback at N = 8); a
    caller stream of another device is NRT_E_INVALID (>= 2 GPUs)."""
    torch = pytest.importorskip("torch")
    with in_golden():
        s = nrt.Scene.load(SCENE, nrt.CameraConfig(width=W, height=H, samples_per_pixel=SPP))
    s.prepare(precision="f32", rng="philox", device=0, gpus=1)
    monkeypatch.setenv("NRT_MULTI_LOOPBACK", "1")
    s.prepare(precision="f32", rng="philox", device=0, gpus=8)
    monkeypatch.delenv("NRT_MULTI_LOOPBACK")
    with pytest.raises(nrt.NrtError):
        s.prepare(device=0, gpus=nrt.device_count() + 1)  # more devices than visible
    if nrt.device_count() >= 2:
        other = torch.cuda.Stream(device=1)
        o = torch.empty((H, W, 3), dtype=torch.float32, device="cuda:0")
        with pytest.raises(nrt.NrtError, match="belongs to device 1"):
            s.render_device(o.data_ptr(), o.numel(), device=0, stream=other.cuda_stream, gpus=1)


@pytest.mark.parametrize("scene,precision,rng", [
    ("scenes/utah-teapot-scene.json", "f32", "philox"),   # world BVH, scene-specialised (BvhSig)
    ("scenes/utah-teapot-scene.json", "f64", "chacha8"),  # the exact kernel's persistent walk, LDS stack
    ("scenes/earth.toml", "f32", "philox"),               # PAL16 textures (KF_TEXPAL), f32 spheres
    ("scenes/spheres.toml", "f64", "chacha8"),            # the unfiltered exact walk (XWalkU)
])
def test_library_multi_gpu_loopback_other_kernels(monkeypatch, scene, precision, rng):
    """The N-GPU render's shards go through every kernel family (loopback, N = 3 and 8, a height that leaves
    short shards): bit-identical to the single-device render."""
    monkeypatch.setenv("NRT_MULTI_LOOPBACK", "1")
    with in_golden():
        s = nrt.Scene.load(scene, nrt.CameraConfig(width=40, height=27, samples_per_pixel=4))
    want = s.render(precision=precision, rng=rng, device=0)
    for g in (3, 8):
        np.testing.assert_array_equal(s.render(precision=precision, rng=rng, device=0, gpus=g), want,
                                      err_msg=f"gpus={g}")
