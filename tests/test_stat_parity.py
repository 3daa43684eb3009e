"""Statistical parity of the fast kernels at the tolerance SURVEY §8(d) states.

The reference estimator is the per-pixel mean of spp path samples
(camera.rs:325-331) with jittered camera rays (camera.rs:250-254).  The f32
and Philox kernels draw other random numbers than the reference's per-pixel
ChaCha8 stream, so their parity is statistical.  The fixtures in
tests/golden/stat/ (scripts/make_stat_fixtures.py) hold the oracle's per-pixel
mean and per-sample variance at a very high spp; against them every variant must
show, per channel,

  * image mean within 0.5 % of the fixture's, and
  * chi^2/N in [0.9, 1.1] for the per-pixel z = (gpu - fixture) / sqrt(var (1/S_gpu + 1/S_fix))
    (Philox: independent streams) or z = (gpu - fixture) / sqrt(var (1/S_gpu - 1/S_fix))
    (ChaCha8: the GPU's S_gpu samples are the first S_gpu of the fixture's own S_fix per
    pixel, so the difference is (1 - S_gpu/S_fix)(first part - remaining part)).

Full-size BASELINE renders (C2 / C4 / C5) cannot be compared pixel by pixel with a
32 x 32 fixture, but a k x k block of a (32k) x (32k) jittered frame integrates
exactly the viewport square of one fixture pixel: the frame mean must be within
0.5 % of the fixture's, and block means are checked against the fixture as a
gross-error guard (chi^2/N <= 1.25; the fine frame is stratified, so its block
variance is at most var / (k^2 spp), but its own heavy-tailed noise dominates).  C5 must also equal its own row shards bit for bit.

Pixels whose fixture variance is zero (rays that always hit the light, k = 1
on a primary hit, diffuse_light.rs:68-72) are compared directly.
"""
import hashlib
import json
import os

import numpy as np
import pytest

from helpers import GOLDEN, in_golden

STAT = os.path.join(GOLDEN, "stat")
MEAN_TOL = 0.005          # per-channel image mean, relative
CHI2 = (0.9, 1.1)         # chi^2 / N window
FULL_CHI2_MAX = 1.25      # full-size block means (conservative statistic, see test_full_size_config)


def manifest():
    with open(os.path.join(STAT, "manifest.json")) as fh:
        return json.load(fh)["cases"]


def fixture(name):
    c = manifest()[name]
    n = c["width"] * c["height"] * 3
    mean = np.fromfile(os.path.join(STAT, c["mean"]), dtype="<f4").astype(np.float64)
    var = np.fromfile(os.path.join(STAT, c["var"]), dtype="<f4").astype(np.float64)
    assert mean.size == n and var.size == n
    return c, mean.reshape(c["height"], c["width"], 3), np.maximum(var, 0.0).reshape(c["height"], c["width"], 3)


def sha256(path):
    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()


def chi2_per_n(got, want, var, factor):
    """(chi^2/N over pixels whose samples vary, max |got - want| over the constant pixels).

    A pixel is constant when its variance is at the rounding level of the oracle's
    (sum of squares - square of sum) form for identical samples."""
    got, want, var = (np.asarray(a, np.float64).reshape(-1) for a in (got, want, var))
    live = var > 1e-9 * np.maximum(want * want, 1e-6)
    z2 = (got[live] - want[live]) ** 2 / (var[live] * factor)
    dead = np.abs(got[~live] - want[~live])
    return float(np.mean(z2)), float(dead.max()) if dead.size else 0.0


def dead_tol(want, s_fix):
    """A pixel that never varied over the fixture's S_fix samples can still hold an event of
    probability below ~3/S_fix (e.g. a grazing hit); allow 10/S_fix of the frame's radiance range."""
    return 10.0 / s_fix * max(1.0, float(np.max(want)))


def channel_rel(got, want):
    g = np.asarray(got, np.float64).reshape(-1, 3).mean(axis=0)
    w = np.asarray(want, np.float64).reshape(-1, 3).mean(axis=0)
    return np.abs(g - w) / np.abs(w)


def block_mean(img, k):
    h, w, _ = img.shape
    return img.astype(np.float64).reshape(h // k, k, w // k, k, 3).mean(axis=(1, 3))


# ------------------------------------------------------------------ CPU: fixtures are intact

def test_stat_fixtures_match_manifest():
    for name, c in manifest().items():
        assert sha256(os.path.join(STAT, c["mean"])) == c["mean_sha256"], name
        assert sha256(os.path.join(STAT, c["var"])) == c["var_sha256"], name
        for f, h in c["inputs"].items():
            assert sha256(os.path.join(GOLDEN, f)) == h, (name, f)
        _, mean, var = fixture(name)
        assert np.all(np.isfinite(mean)) and np.all(mean >= 0) and np.all(var >= 0)
        np.testing.assert_allclose(mean.reshape(-1, 3).mean(axis=0), c["channel_mean"], rtol=1e-6)


def test_statistics_detect_a_one_percent_bias():
    """The statistics themselves: unbiased Gaussian draws pass both; a 1 % bias fails both (the mean
    test alone already sees 0.5 %: 32 x 32 pixels of the Cornell box's heavy-tailed light paths)."""
    _, mean, var = fixture("cornell_32")
    s_gpu, s_fix = 262144, manifest()["cornell_32"]["spp"]
    rng = np.random.default_rng(1)
    draw = mean + rng.standard_normal(mean.shape) * np.sqrt(var * (1 / s_gpu + 1 / s_fix))
    c2, _ = chi2_per_n(draw, mean, var, 1 / s_gpu + 1 / s_fix)
    assert CHI2[0] <= c2 <= CHI2[1], c2
    assert np.all(channel_rel(draw, mean) < MEAN_TOL)
    c2b, _ = chi2_per_n(draw * 1.01, mean, var, 1 / s_gpu + 1 / s_fix)
    assert c2b > CHI2[1], c2b
    assert np.all(channel_rel(draw * 1.01, mean) > MEAN_TOL)


# ------------------------------------------------------------------ GPU

def load(scene, w, h, spp):
    import nrt

    with in_golden():
        return nrt.Scene.load(scene, nrt.CameraConfig(width=w, height=h, samples_per_pixel=spp))


VARIANTS = [
    # (fixture, precision, rng, trace, spp on the GPU)
    ("cornell_32", "f32", "philox", "auto", 262144),       # the headline kernel (world list)
    ("cornell_32", "f32", "philox", "bvh", 262144),        # instance BVH
    ("cornell_32", "f32", "philox", "world-bvh", 262144),  # world BVH
    ("cornell_32", "f64", "philox", "auto", 65536),
    ("cornell_32", "f32", "chacha8", "auto", 16384),       # reference stream, f32 arithmetic
    ("teapot_32", "f32", "philox", "auto", 65536),         # world BVH (C4's kernel)
    ("teapot_32", "f32", "philox", "bvh", 16384),
    ("teapot_32", "f64", "philox", "auto", 16384),
    ("earth_48", "f32", "philox", "auto", 65536),         # image textures, f32 spheres (r = 1000 ground)
    ("earth_48", "f32", "chacha8", "auto", 4096),
]


@pytest.mark.gpu
@pytest.mark.parametrize("name,precision,rng,trace,spp", VARIANTS,
                         ids=[f"{v[0]}-{v[1]}-{v[2]}-{v[3]}" for v in VARIANTS])
def test_variant_within_stated_tolerance(name, precision, rng, trace, spp):
    c, want, var = fixture(name)
    s = load(c["scene"], c["width"], c["height"], spp)
    got = s.render(precision=precision, rng=rng, trace=trace).astype(np.float64)
    assert np.all(np.isfinite(got)) and np.all(got >= 0)
    rel = channel_rel(got, want)
    assert np.all(rel < MEAN_TOL), f"per-channel mean off by {rel}"
    if rng == "chacha8":
        assert spp < c["spp"]
        factor = 1.0 / spp - 1.0 / c["spp"]
    else:
        factor = 1.0 / spp + 1.0 / c["spp"]
    c2, dead = chi2_per_n(got, want, var, factor)
    print(f"{name} {precision}/{rng}/{trace} spp={spp}: chi2/N = {c2:.4f}, mean rel {rel}, constant-pixel max diff {dead:.2e}")
    assert CHI2[0] <= c2 <= CHI2[1], f"chi2/N = {c2:.4f}"
    assert dead <= dead_tol(want, c["spp"]), dead


@pytest.mark.gpu
def test_f32_chacha8_pixels_follow_the_reference_stream():
    """SURVEY §8(d) f32 + ChaCha8 rule: >= 95 % of pixels within max(2e-3, 3 sigma/sqrt(spp)) of the
    oracle at the same spp (same per-pixel stream), per-channel mean within 0.5 %."""
    import tempfile

    from helpers import oracle_render, oracle_tree

    scene, w, h, spp = "scenes/cornell-box-scene.json", 48, 40, 64
    with tempfile.TemporaryDirectory() as td:
        tree, _ = oracle_tree(scene, td, width=w, height=h, spp=spp)
        want, _, var = oracle_render(tree, var=True)
    got = load(scene, w, h, spp).render(precision="f32", rng="chacha8").reshape(-1).astype(np.float64)
    want = want.astype(np.float64)
    tol = np.maximum(2e-3, 3.0 * np.sqrt(np.maximum(var, 0.0)) / np.sqrt(spp))
    ok = np.abs(got - want) <= tol
    assert np.mean(ok) >= 0.95, np.mean(ok)
    assert np.all(channel_rel(got, want) < MEAN_TOL)


FULL = [
    # (config, fixture, scene, W, H, spp, trace)
    ("C5", "cornell_32", "scenes/cornell-box-scene.json", 1024, 1024, 256, "auto"),
    ("C2", "cornell_32", "scenes/cornell-box-scene.json", 512, 512, 64, "auto"),
    ("C4", "teapot_32", "scenes/utah-teapot-scene.json", 1024, 1024, 256, "auto"),
    ("C3", "earth_48", "scenes/earth.toml", 1920, 1080, 128, "auto"),
]


@pytest.mark.gpu
@pytest.mark.parametrize("cfg,name,scene,w,h,spp,trace", FULL, ids=[f[0] for f in FULL])
def test_full_size_config(cfg, name, scene, w, h, spp, trace):
    c, want, var = fixture(name)
    k = w // c["width"]
    assert k * c["width"] == w and k * c["height"] == h
    s = load(scene, w, h, spp)
    img = s.render(precision="f32", rng="philox", trace=trace)
    assert img.shape == (h, w, 3)
    assert np.all(np.isfinite(img)) and np.all(img >= 0)
    rel = channel_rel(img, want)
    assert np.all(rel < MEAN_TOL), f"{cfg}: per-channel frame mean off by {rel}"
    blocks = block_mean(img, k)
    c2, dead = chi2_per_n(blocks, want, var, 1.0 / (k * k * spp) + 1.0 / c["spp"])
    print(f"{cfg}: block chi2/N = {c2:.4f}, frame mean rel {rel}, constant-block max diff {dead:.2e}")
    # a gross-error guard: at these sizes the fine frame's own noise dominates the statistic
    # (C2: 16 384 samples per block) and heavy-tailed light paths spread it; the sharp
    # per-pixel statistics are the 32 x 32 tests above, the sharp full-size one the mean
    assert c2 <= FULL_CHI2_MAX, f"{cfg}: block chi2/N = {c2:.4f}"
    assert dead <= dead_tol(want, c["spp"]), dead
    if cfg == "C5":  # the multi-GPU partition: any row shard reproduces its rows bit for bit
        for stride in (2, 4, 8):
            for off in range(stride):
                part = s.render(precision="f32", rng="philox", trace=trace, row_offset=off, row_stride=stride)
                np.testing.assert_array_equal(part, img[off::stride], err_msg=f"stride {stride} offset {off}")
