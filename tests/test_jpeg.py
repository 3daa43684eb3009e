"""Image texture decoding (Image::try_from_path -> into_rgb32f, lib/textures/image.rs:24-28).

The reference decodes with image 0.25.8 / zune-jpeg 0.4.21 (absent here); the
library's decoder follows libjpeg's islow IDCT and YCbCr tables, so it is
checked bit for bit against PIL (libjpeg-turbo) -- the decoder the oracle's
loader uses.  Parity with zune-jpeg itself is unpinned.
"""
import io
import os

import numpy as np
import pytest

import nrt
from helpers import GOLDEN

Image = pytest.importorskip("PIL.Image")


def pil_rgb32f(path):
    return np.asarray(Image.open(path).convert("RGB"), dtype=np.uint8).astype(np.float32) / np.float32(255.0)


@pytest.mark.parametrize("name", ["earth.jpg", "moon.jpg"])
def test_reference_textures_match_libjpeg(name):
    path = os.path.join(GOLDEN, "scenes", "textures", name)
    got = nrt.image_load(path)
    assert got.shape == (1024, 2048, 3)
    np.testing.assert_array_equal(got, pil_rgb32f(path))


def _synthetic(w, h, mode="RGB", seed=0):
    rng = np.random.default_rng(seed)
    yy, xx = np.mgrid[0:h, 0:w]
    base = np.stack([(xx * 255 // max(w - 1, 1)), (yy * 255 // max(h - 1, 1)), ((xx + yy) * 7) % 256], -1)
    img = np.clip(base + rng.integers(-40, 40, size=base.shape), 0, 255).astype(np.uint8)
    return Image.fromarray(img[..., 0] if mode == "L" else img, mode)


@pytest.mark.parametrize("w,h,kw", [
    (64, 48, dict(quality=90, subsampling=0)),
    (37, 23, dict(quality=75, subsampling=0)),            # partial edge blocks
    (100, 60, dict(quality=50, subsampling=0, restart_marker_blocks=3)),  # restart intervals
    (16, 16, dict(quality=100, subsampling=0)),
    (33, 17, dict(quality=95, subsampling=0, optimize=True)),  # optimised Huffman tables
])
def test_synthetic_444_bit_exact(tmp_path, w, h, kw):
    p = tmp_path / "t.jpg"
    _synthetic(w, h).save(p, "JPEG", **kw)
    np.testing.assert_array_equal(nrt.image_load(str(p)), pil_rgb32f(p))


def test_grayscale_bit_exact(tmp_path):
    p = tmp_path / "g.jpg"
    _synthetic(41, 29, mode="L").save(p, "JPEG", quality=80)
    got = nrt.image_load(str(p))
    np.testing.assert_array_equal(got, pil_rgb32f(p))
    assert np.array_equal(got[..., 0], got[..., 1]) and np.array_equal(got[..., 1], got[..., 2])


def test_subsampled_close(tmp_path):
    # 4:2:0: chroma replicated instead of libjpeg's triangle filter -> small differences only
    yy, xx = np.mgrid[0:40, 0:64]
    smooth = np.stack([xx * 4, yy * 6, (xx + yy) * 2], -1).clip(0, 255).astype(np.uint8)
    for ss in (1, 2):  # 4:2:2, 4:2:0
        p = tmp_path / f"s{ss}.jpg"
        Image.fromarray(smooth).save(p, "JPEG", quality=95, subsampling=ss)
        d = np.abs(nrt.image_load(str(p)) - pil_rgb32f(p)) * 255
        assert d.max() <= 8 and d.mean() < 2.0, (ss, d.max(), d.mean())


def test_progressive_and_garbage_rejected(tmp_path):
    p = tmp_path / "p.jpg"
    _synthetic(32, 32).save(p, "JPEG", progressive=True)
    with pytest.raises(nrt.NrtError) as ei:
        nrt.image_load(str(p))
    assert ei.value.code == -2 and "progressive" in str(ei.value).lower() or "baseline" in str(ei.value).lower()
    q = tmp_path / "bad.jpg"
    q.write_bytes(b"\xff\xd8\xff\xdb\x00\x04\x00")
    with pytest.raises(nrt.NrtError):
        nrt.image_load(str(q))
    with pytest.raises(nrt.NrtError):
        nrt.image_load(str(tmp_path / "missing.jpg"))
