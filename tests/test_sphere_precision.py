"""Sphere precision classes of the f32 world modes (flatten.cpp, kernel.hpp sphere_t_world_f32).

A sphere whose anchor P (its point nearest the world origin) lies within the scene scale takes the
f32 quadratic relative to P at any radius (the r = 1000 ground sphere of spheres.toml / earth.toml
included) and its hit point the anchored Newton step back onto the surface; a sphere anchored
outside that scale keeps the f64 quadratic in the world list, and leaves its scene to the
instance BVH instead of the world BVH (whose leaves compile the f32 test only).  The reference
intersects every sphere in f64 (sphere.rs:105-163): the f32 kernels must follow the exact kernel's
paths on the same ChaCha8 stream at few bounces, as tests/test_gpu_parity.py's
test_fast_kernel_follows_exact_paths asks of the reference scenes.
"""
import numpy as np
import pytest

import nrt

W, H = 40, 28
CAM = dict(width=W, height=H, background_color=(0.7, 0.8, 1.0), look_from=(0.0, 2.0, 7.0), look_at=(0.0, 0.5, 0.0),
           view_up=(0.0, 1.0, 0.0), defocus_angle=0.0, focus_dist=1.0, field_of_view=0.7)
NEAR = [((0.0, -1000.0, 0.0), 1000.0, 3), ((-1.2, 0.5, 0.0), 0.5, 0), ((0.0, 0.5, 0.0), 0.5, 1), ((1.2, 0.5, 0.0), 0.5, 2)]
# a large sphere anchored ~200 units out (|P| + |speed| > 100): f64 in the world list
FAR = [((0.0, 0.0, -260.0), 60.0, 0)]


def scene(spheres, bounces, spp=1):
    b = nrt.Builder()
    red, grey = b.solid((0.8, 0.2, 0.1)), b.solid((0.5, 0.5, 0.5))
    mats = [b.lambertian(red), b.metal(0.1, b.solid((0.8, 0.8, 0.9))), b.dielectric(1.5), b.lambertian(grey)]
    objs = [b.sphere(c, r, mats[m]) for c, r, m in spheres]
    cam = nrt.CameraBuilder(samples_per_pixel=spp, ray_max_bounces=bounces, **CAM).build()
    return b.finish(b.bvh(objs), cam)


def mismatch(a, b):
    return np.mean(np.abs(a - b).max(axis=2) > 1e-3 + 1e-3 * np.abs(b).max(axis=2))


@pytest.mark.gpu
@pytest.mark.parametrize("bounces", [1, 2, 3])
@pytest.mark.parametrize("trace", ["world-list", "world-bvh"])
def test_anchored_f32_spheres_follow_exact_paths(bounces, trace):
    """Every sphere here is anchored within the scene scale (the ground's anchor is the origin):
    both world modes test them in f32 and must trace the exact kernel's paths."""
    s = scene(NEAR, bounces)
    a = s.render(precision="f32", rng="chacha8", trace=trace)
    b = s.render(precision="f64", rng="chacha8")
    assert mismatch(a, b) <= 0.01, mismatch(a, b)


def test_far_anchored_sphere_keeps_the_exact_culling_walk():
    """The far sphere bars only the f32 world-BVH kernels (their leaves hold the f32 test); the
    tree is still built, so the reference-exact kernel keeps its world-BVH culling walk, which
    tests every primitive it reaches in f64 (nrt.h NRT_EXACT_WORLD = 2)."""
    assert scene(NEAR + FAR, 2).stats()["exact_mode"] == 2
    assert scene(NEAR, 2).stats()["exact_mode"] == 2


@pytest.mark.gpu
@pytest.mark.parametrize("bounces", [1, 2])
def test_far_anchored_sphere_stays_f64(bounces):
    """A sphere anchored outside the scene scale: the world list tests it in f64 beside the f32
    ones (and follows the exact paths), the world BVH is not offered for the scene (its leaves
    hold the f32 test only), and AUTO renders it through the instance BVH."""
    s = scene(NEAR + FAR, bounces)
    assert s.stats()["world_list_ok"]
    with pytest.raises(nrt.NrtError):
        s.render(precision="f32", rng="chacha8", trace="world-bvh")
    b = s.render(precision="f64", rng="chacha8")
    for trace in ("world-list", "auto"):
        a = s.render(precision="f32", rng="chacha8", trace=trace)
        assert mismatch(a, b) <= 0.01, (trace, mismatch(a, b))
