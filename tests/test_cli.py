"""`nrt-cli render` (the reference's `render` command, app/commands/render.rs:104-115, cli.rs:111-270).

`--legacy-schema` is a switch (no value): it loads the index schema of scenes/triangles.toml
(NRT_LOAD_LEGACY_SCHEMA), which the default loader rejects as the reference's does.  CPU: the
load decision (without the switch the scene fails to load; with it the run gets past the load and
stops only for want of a GPU).  GPU: the PFM the CLI writes equals the library's render of the same
scene and camera, bit for bit.
"""
import os
import subprocess

import numpy as np
import pytest

import nrt
from helpers import in_golden

CLI = os.path.join(os.path.dirname(nrt.LIB_PATH), "nrt-cli")
GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")


def run(args, tmp_path, extra_env=None):
    env = dict(os.environ)
    for k in list(env):
        if k.startswith("NR_RT_CAMERA_"):
            del env[k]
    env.update(extra_env or {})
    return subprocess.run([CLI, "render", *args], cwd=GOLDEN, capture_output=True, text=True, env=env, timeout=300)


def read_pfm(path):
    with open(path, "rb") as fh:
        assert fh.readline().strip() == b"PF"
        w, h = (int(x) for x in fh.readline().split())
        assert float(fh.readline()) < 0  # little endian
        data = np.frombuffer(fh.read(), dtype="<f4").reshape(h, w, 3)
    return data[::-1]  # PFM rows run bottom to top


def test_legacy_schema_refused_without_the_switch(tmp_path):
    out = tmp_path / "t.pfm"
    r = run(["scenes/triangles.toml", "-W", "16", "-H", "12", "-o", str(out), "-f"], tmp_path)
    assert r.returncode != 0
    assert "unknown flag" not in r.stderr
    assert "GPUs" not in r.stderr and "visible" not in r.stderr, r.stderr  # it failed at the load


def test_legacy_schema_switch_takes_no_value(tmp_path):
    # the switch before the scene path: the path must stay the scene (round-3 ADVICE: the switch once
    # swallowed it as its value)
    out = tmp_path / "t.pfm"
    r = run(["--legacy-schema", "scenes/triangles.toml", "-W", "16", "-H", "12", "-o", str(out), "-f"], tmp_path)
    if nrt.device_count() < 1:
        assert r.returncode != 0 and "visible" in r.stderr, r.stderr  # loaded; no GPU to render on
    else:
        assert r.returncode == 0, r.stderr


@pytest.mark.gpu
@pytest.mark.parametrize("args,precision,rng", [([], "f64", "chacha8"),
                                                (["--precision", "f32", "--rng", "philox"], "f32", "philox")])
def test_cli_pfm_equals_library_render(tmp_path, args, precision, rng):
    out = tmp_path / "t.pfm"
    r = run(["--legacy-schema", "scenes/triangles.toml", "-W", "40", "-H", "30", "--samples-per-pixel", "4",
             "-o", str(out), "-f", *args], tmp_path)
    assert r.returncode == 0, r.stderr
    got = read_pfm(out)
    with in_golden():
        s = nrt.Scene.load("scenes/triangles.toml", nrt.CameraConfig(width=40, height=30, samples_per_pixel=4),
                           legacy_schema=True)
    want = s.render(precision=precision, rng=rng)
    np.testing.assert_array_equal(got.view(np.uint32), want.view(np.uint32))


@pytest.mark.gpu
def test_cli_multi_gpu_rows_equal_single_gpu(tmp_path):
    """`--gpus N` is the library's multi-GPU render (nrt_render_opts.gpus, csrc/multi.hip): rows
    y = g (mod N) on device g, one RCCL gather to device 0, un-permuted there; every device runs the
    scene-specialised kernel or, failing that, the generic one, which renders the same bits, so the
    frame equals the one-GPU frame."""
    n = nrt.device_count()
    if n < 2:
        pytest.skip("needs two GPUs")
    outs = []
    for g in (1, min(n, 4)):
        out = tmp_path / f"g{g}.pfm"
        r = run(["scenes/cornell-box-scene.json", "-W", "64", "-H", "48", "--samples-per-pixel", "8", "--precision",
                 "f32", "--rng", "philox", "--gpus", str(g), "-o", str(out), "-f"], tmp_path)
        assert r.returncode == 0, r.stderr
        outs.append(read_pfm(out))
    np.testing.assert_array_equal(outs[0].view(np.uint32), outs[1].view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("precision,rng", [("f32", "philox"), ("f64", "chacha8")])
def test_cli_multi_gpu_code_on_one_gpu(tmp_path, precision, rng):
    """`--gpus 3` on one GPU: the library's N-GPU render through the test-only loopback (NRT_MULTI_LOOPBACK=1:
    the three shards on device 0, the gather as device copies, csrc/multi.hip), and the CLI's own fallback
    for a host without a usable librccl (NRT_CLI_SHARDS=1: one thread per shard, rows y = g (mod 3), the
    frame un-permuted on the host, as nrt_render_prepare's NRT_E_UNSUPPORTED makes it): both PFMs equal the
    one-GPU render bit for bit."""
    args = ["scenes/cornell-box-scene.json", "-W", "40", "-H", "29", "--samples-per-pixel", "4", "--precision",
            precision, "--rng", rng, "-f"]
    outs = []
    for name, gpus, env in (("one", 1, {}), ("loop", 3, {"NRT_MULTI_LOOPBACK": "1"}),
                            ("shards", 3, {"NRT_MULTI_LOOPBACK": "1", "NRT_CLI_SHARDS": "1"})):
        out = tmp_path / f"{name}.pfm"
        r = run(args + ["--gpus", str(gpus), "-o", str(out)], tmp_path, env)
        assert r.returncode == 0, (name, r.stderr)
        outs.append(read_pfm(out))
    np.testing.assert_array_equal(outs[1].view(np.uint32), outs[0].view(np.uint32))
    np.testing.assert_array_equal(outs[2].view(np.uint32), outs[0].view(np.uint32))
