"""Image texel formats (device_scene.hpp TEXFMT_*): every file image is k / 255 per channel
(into_rgb32f, textures/image.rs:24-28), stored as PAL16 (a 16-bit palette index per texel plus a
palette of at most 65536 RGBA8 words per band of rows) when its colours allow, else as 3-byte
RGB8T texels (knob NRT_TEX_PAL=0), and decoded back to exactly k / 255.0 either way.

CPU: earth.toml's two textures take PAL16 (2 bytes per texel plus palettes instead of 3.2).
GPU: the f64 / ChaCha8 and f32 / Philox frames are the same bit for bit in both formats (the
kernels read the same texel values; only the fetch differs).
"""
import numpy as np
import pytest

import nrt
from helpers import in_golden


def load(w=48, h=27, spp=4):
    with in_golden():
        return nrt.Scene.load("scenes/earth.toml", nrt.CameraConfig(width=w, height=h, samples_per_pixel=spp))


def test_earth_textures_take_the_palette_format(monkeypatch):
    pal = load().stats()
    monkeypatch.setenv("NRT_TEX_PAL", "0")
    rgb8 = load().stats()
    assert pal["texels"] == rgb8["texels"] == 2 * 2048 * 1024
    assert rgb8["texel_bytes"] / rgb8["texels"] == pytest.approx(3.2, rel=0.01)  # 8 x 5 tiles of 128 B
    # 2 B per texel in 8 x 8 tiles, plus one 65536-word palette per band (earth 4 bands, moon 1)
    assert pal["texel_bytes"] == 2 * 2048 * 1024 * 2 + 5 * 65536 * 4


@pytest.mark.gpu
@pytest.mark.parametrize("precision,rng", [("f64", "chacha8"), ("f32", "philox")])
def test_palette_and_rgb8_frames_bitwise_identical(monkeypatch, precision, rng):
    a = load().render(precision=precision, rng=rng)
    monkeypatch.setenv("NRT_TEX_PAL", "0")
    b = load().render(precision=precision, rng=rng)
    assert np.isfinite(a).all() and a.max() > 0
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
