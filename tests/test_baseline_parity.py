"""Reference-exact parity at the BASELINE.json configurations' own sizes.

The reference renders pixel after pixel, each from its own ChaCha8 stream (`set_stream(pixel
index)`) drawn through ALL its spp samples in order (camera.rs:318-331).  At C5 / C4's 1024 x 1024,
spp 256 a pixel's last draws sit ~1 600 blocks into a stream whose index reaches 2^20 - 1 (C3:
2^21), far past the small cases of tests/test_gpu_parity.py (<= 64 x 40, spp <= 8).  Here:

  * the f64 / ChaCha8 kernel renders each configuration's committed oracle row sample
    (tests/golden/baseline/, scripts/make_baseline_fixtures.py: full image size and spp, rows
    y = (H - 1) mod stride (mod stride), so the frame's last row is in it) through the C ABI
    (nrt_render_opts row_offset / row_stride): >= 99.9 % of values bit-identical, max relative
    error <= 1e-6 (the bar of test_gpu_parity.py);
  * the kernel's stream probe at block ~1 600 of pixel streams up to 2^20 - 1, against an
    independent Python ChaCha8 (RFC 7539 block, pinned in tests/test_oracle.py);
  * (CPU) the fixtures' sha256 manifest, and the oracle re-rendering two of them byte for byte.
"""
import hashlib
import json
import os
import subprocess
import tempfile

import numpy as np
import pytest

from helpers import GOLDEN, ORACLE_BIN, ensure_oracle, in_golden, oracle_render, oracle_tree

BASE = os.path.join(GOLDEN, "baseline")
with open(os.path.join(BASE, "manifest.json")) as _fh:
    MANIFEST = json.load(_fh)["cases"]


def _sha(path):
    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()


def _fixture(name):
    c = MANIFEST[name]
    img = np.fromfile(os.path.join(BASE, c["image"]), dtype="<f4")
    assert img.size == c["rows"] * c["width"] * 3
    return c, img


def test_baseline_fixtures_manifest():
    """Every fixture and every scene input it was rendered from match the manifest's sha256."""
    assert set(MANIFEST) == {"c1_spheres", "c2_cornell", "c3_earth", "c4_teapot", "c5_cornell"}
    for name, c in MANIFEST.items():
        assert _sha(os.path.join(BASE, c["image"])) == c["image_sha256"], name
        for f, h in c["inputs"].items():
            assert _sha(os.path.join(GOLDEN, f)) == h, (name, f)
        assert c["max_pixel_index"] == c["width"] * c["height"] - 1, name  # the last row is sampled


@pytest.mark.parametrize("name", ["c2_cornell", "c5_cornell"])
def test_oracle_reproduces_baseline_fixture(name):
    """The committed rows are what the oracle renders now (C5: 4.2 M samples, ~2 s on 8 cores)."""
    c, want = _fixture(name)
    with tempfile.TemporaryDirectory() as td:
        tree, _ = oracle_tree(c["scene"], td, width=c["width"], height=c["height"], spp=c["spp"])
        got, _ = oracle_render(tree, threads=os.cpu_count(), rows=(c["row_offset"], c["row_stride"]))
    assert got.tobytes() == want.tobytes()


def py_stream_at(stream, first, count):
    """Draws first .. first + count - 1 of rand_chacha's BlockRng<ChaCha8Core> stream (u64 = lo | hi << 32;
    draw i uses words 2i, 2i + 1 of the keystream, block (2i) // 16), computing only the blocks needed."""
    from test_oracle import pcg32_key, py_chacha_block
    key = pcg32_key(0)
    b0, b1 = (2 * first) // 16, (2 * (first + count) - 1) // 16
    words = []
    for b in range(b0, b1 + 1):
        words += py_chacha_block(8, key, b, stream)
    base = 2 * first - 16 * b0
    return [words[base + 2 * i] | (words[base + 2 * i + 1] << 32) for i in range(count)]


def test_oracle_deep_stream_matches_python_chacha8():
    """The oracle's generator (oracle.cpp's BlockRng) at block ~1 600 of pixel stream 2^20 - 1."""
    ensure_oracle()
    n = 12864
    r = subprocess.run([ORACLE_BIN, "rng", str(2 ** 20 - 1), str(n)], check=True, capture_output=True, text=True)
    got = [int(x, 16) for x in r.stdout.split()]
    assert len(got) == n
    assert got[-64:] == py_stream_at(2 ** 20 - 1, n - 64, 64)


@pytest.mark.gpu
def test_chacha8_stream_deep_matches_python():
    """The kernel's ChaCha8 (kernel.hpp, LDS ring and refills) at draws 12 800 .. 12 863 (keystream
    block 1 600 and on) of pixel streams 2^20 - 64 .. 2^20 - 1: the depth C5's spp 256 reaches."""
    import nrt
    n, first = 12864, 12800
    got = nrt.debug_rng("chacha8", 2 ** 20 - 64, 64, n)
    for lane in (0, 31, 63):
        assert got[lane, first:].tolist() == py_stream_at(2 ** 20 - 64 + lane, first, n - first), lane


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_f64_chacha8_matches_oracle_at_baseline_size(name):
    import nrt
    c, want = _fixture(name)
    with in_golden():
        s = nrt.Scene.load(c["scene"], nrt.CameraConfig(width=c["width"], height=c["height"],
                                                        samples_per_pixel=c["spp"]))
    got = s.render(precision="f64", rng="chacha8", device=0, row_offset=c["row_offset"],
                   row_stride=c["row_stride"]).reshape(-1)
    assert got.shape == want.shape
    assert np.all(np.isfinite(got))
    same = float(np.mean(got == want))
    rel = np.abs(got.astype(np.float64) - want) / np.maximum(np.abs(want.astype(np.float64)), 1e-30)
    assert same >= 0.999, f"{name}: bit-identical fraction {same:.5f}"
    assert float(np.max(rel)) <= 1e-6, f"{name}: max rel err {np.max(rel):.3e}"
