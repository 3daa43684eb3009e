"""Image texel formats (device_scene.hpp TEXFMT_*): every file image is k / 255 per channel
(into_rgb32f, textures/image.rs:24-28), stored as PAL16 (a 16-bit palette index per texel plus a
palette of at most 65536 RGBA8 words per band of rows) when its colours allow, else as 3-byte
RGB8T texels (knob NRT_TEX_PAL=0), and decoded back to exactly k / 255.0 either way.  The band
palettes sit 2^p words apart (the largest band's colour count rounded up to a power of two), and
PAL16 is taken only where index + palettes are smaller than RGB8T.

CPU: earth.toml's two textures take PAL16 (2 bytes per texel plus palettes instead of 3.2); a small
image takes PAL16 with a small palette when it has few colours and RGB8T when it has many.
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
    # 2 B per texel in 8 x 8 tiles, plus per band a palette 2^p words apart: earth 4 bands of <= 62 033
    # colours (2^16), moon 1 band of 10 532 (2^14)
    assert pal["texel_bytes"] == 2 * 2048 * 1024 * 2 + (4 * 65536 + 16384) * 4
    assert pal["texel_formats"] == 1 << 3 and rgb8["texel_formats"] == 1 << 2


def small_image_scene(colours, spp=4, w=64, h=64):
    """A sphere textured with a w x h image of `colours` distinct k / 255 colours, under a light."""
    rng = np.random.default_rng(7)
    pal = rng.integers(0, 256, size=(colours, 3))
    img = (pal[rng.integers(0, colours, size=(h, w))] / 255.0).astype(np.float32)
    b = nrt.Builder()
    tex = b.image(img)
    objs = [b.sphere((0.0, 0.0, 0.0), 1.0, b.lambertian(tex)),
            b.sphere((0.0, -101.0, 0.0), 100.0, b.lambertian(b.solid((0.5, 0.5, 0.5))))]
    cam = nrt.CameraBuilder(width=40, height=30, samples_per_pixel=spp, background_color=(0.7, 0.8, 1.0),
                            look_from=(0.0, 0.5, 4.0), look_at=(0.0, 0.0, 0.0), field_of_view=0.7,
                            ray_max_bounces=8).build()
    return b.finish(b.bvh(objs), cam)


def test_small_image_palette_sized_to_its_colours():
    few = small_image_scene(16).stats()
    assert few["texel_formats"] == 1 << 3  # PAL16: 64 x 64 indices (8 KB) + a 16-word palette
    assert few["texel_bytes"] == 64 * 64 * 2 + 16 * 4
    many = small_image_scene(4000).stats()  # 4000 colours: index + 4096-word palette > RGB8T's 13 KB
    assert many["texel_formats"] == 1 << 2
    assert many["texel_bytes"] == 8 * 13 * 128


@pytest.mark.gpu
@pytest.mark.parametrize("precision,rng", [("f64", "chacha8"), ("f32", "philox")])
def test_small_palette_frames_match_rgb8(monkeypatch, precision, rng):
    a = small_image_scene(16).render(precision=precision, rng=rng)
    monkeypatch.setenv("NRT_TEX_PAL", "0")
    b = small_image_scene(16).render(precision=precision, rng=rng)
    assert np.isfinite(a).all() and a.max() > 0
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))


@pytest.mark.gpu
@pytest.mark.parametrize("precision,rng", [("f64", "chacha8"), ("f32", "philox")])
def test_palette_and_rgb8_frames_bitwise_identical(monkeypatch, precision, rng):
    a = load().render(precision=precision, rng=rng)
    monkeypatch.setenv("NRT_TEX_PAL", "0")
    b = load().render(precision=precision, rng=rng)
    assert np.isfinite(a).all() and a.max() > 0
    np.testing.assert_array_equal(a.view(np.uint32), b.view(np.uint32))
