"""Moving spheres: SphereBuilder::with_speed (lib/objects/sphere.rs:45-50, box over both end
positions sphere.rs:69-92) and the centre Ray::new(center, speed).at(time) (sphere.rs:110-111),
the only consumer of the camera ray's `time` draw (camera.rs:264).  No reference scene file has
a moving sphere (scene_config.rs builds spheres without a speed), so the scene is built through
the constructor API (nrt_object_sphere_moving) and, independently, as an oracle tree.

CPU: the product's graph (boxes, centres, speeds) equals the oracle's.
GPU: the f64 / ChaCha8 kernel against the oracle (>= 99.9 % of values bit-identical, max
relative error 1e-6, as tests/test_gpu_parity.py), and the f32 / Philox kernels of every
traversal against the oracle's image at the same spp (per-channel means within 4.5 standard
errors, block z-scores as test_fast_variants_statistically_match).
"""
import os
import tempfile

import numpy as np
import pytest

import nrt
from helpers import oracle_dump, oracle_render

W, H = 48, 32
CAM = dict(width=W, height=H, background_color=(0.7, 0.8, 1.0), look_from=(0.0, 1.5, 6.0), look_at=(0.0, 0.5, 0.0),
           view_up=(0.0, 1.0, 0.0), defocus_angle=0.0, focus_dist=1.0, field_of_view=0.6981317007977318,
           ray_max_bounces=10)
# (centre, radius, speed or None, material index): materials 0 lambertian red, 1 metal, 2 glass, 3 grey ground
SPHERES = [
    ((0.0, -1000.0, 0.0), 1000.0, None, 3),
    ((-1.6, 0.5, 0.0), 0.5, (0.0, 0.6, 0.0), 0),
    ((0.0, 0.5, -0.5), 0.5, (0.7, 0.0, 0.0), 1),
    ((1.6, 0.5, 0.0), 0.5, (0.0, 0.0, 1.2), 2),
    ((0.6, 0.3, 1.4), 0.3, (-0.5, 0.25, 0.0), 0),
    ((-0.7, 0.25, 1.6), 0.25, None, 1),
]


def _f(x):
    return float(x).hex()


def build_product(spp):
    b = nrt.Builder()
    red, grey = b.solid((0.8, 0.2, 0.1)), b.solid((0.5, 0.5, 0.5))
    mats = [b.lambertian(red), b.metal(0.1, b.solid((0.8, 0.8, 0.9))), b.dielectric(1.5), b.lambertian(grey)]
    objs = [b.sphere(c, r, mats[m], speed=s) for c, r, s, m in SPHERES]
    cam = nrt.CameraBuilder(samples_per_pixel=spp, **CAM).build()
    return b.finish(b.bvh(objs), cam)


def oracle_tree_text(spp):
    c = CAM
    lines = [f"CAMERA {c['width']} {c['height']} {spp} {c['ray_max_bounces']} "
             + " ".join(_f(x) for x in (*c["background_color"], *c["look_from"], *c["look_at"], *c["view_up"]))
             + f" {_f(c['defocus_angle'])} {_f(c['focus_dist'])} {_f(c['field_of_view'])}",
             "TEX 0 SOLID " + " ".join(_f(x) for x in (0.8, 0.2, 0.1)),
             "TEX 1 SOLID " + " ".join(_f(x) for x in (0.5, 0.5, 0.5)),
             "TEX 2 SOLID " + " ".join(_f(x) for x in (0.8, 0.8, 0.9)),
             "MAT 0 LAMBERTIAN 0", f"MAT 1 METAL {_f(0.1)} 2", f"MAT 2 DIELECTRIC {_f(1.5)}", "MAT 3 LAMBERTIAN 1"]
    for i, (ctr, r, s, m) in enumerate(SPHERES):
        speed = "" if s is None else " " + " ".join(_f(x) for x in s)
        lines.append(f"OBJ {i} SPHERE " + " ".join(_f(x) for x in (*ctr, r)) + f" {m}" + speed)
    n = len(SPHERES)
    lines += [f"OBJ {n} BVH {n} " + " ".join(str(i) for i in range(n)), f"ROOT {n}"]
    return "\n".join(lines) + "\n"


def oracle_image(spp, var=False):
    with tempfile.TemporaryDirectory() as td:
        tree = os.path.join(td, "moving.tree")
        with open(tree, "w") as fh:
            fh.write(oracle_tree_text(spp))
        return oracle_render(tree, var=var)


def _norm(text):
    out = []
    for line in text.splitlines()[1:]:  # the object graph (the camera lines are spelled differently)
        toks = []
        for t in line.split():
            toks.append(repr(float.fromhex(t)) if t.startswith(("0x", "-0x")) else t)
        out.append(" ".join(toks))
    return out


def test_moving_sphere_graph_matches_oracle():
    got = "CAMERA\n" + build_product(4).dump()
    with tempfile.TemporaryDirectory() as td:
        tree = os.path.join(td, "moving.tree")
        with open(tree, "w") as fh:
            fh.write(oracle_tree_text(4))
        want = oracle_dump(tree)
    a, b = _norm(got), _norm(want)
    assert len(a) == len(b) and any("SPHERE" in x for x in a)
    for i, (x, y) in enumerate(zip(a, b)):
        assert x == y, f"line {i}:\nproduct {x}\noracle  {y}"


def test_moving_sphere_speed_reaches_the_graph():
    # the box spans the centre at time 0 and time 1 (sphere.rs:72-84): a speed must change the dump
    b = nrt.Builder()
    m = b.lambertian(b.solid((1, 1, 1)))
    still = b.finish(b.bvh([b.sphere((0, 0, 0), 1.0, m)])).dump()
    moving = b.finish(b.bvh([b.sphere((0, 0, 0), 1.0, m, speed=(2.0, 0.0, 0.0))])).dump()
    assert still != moving


@pytest.mark.gpu
def test_moving_sphere_f64_chacha8_matches_oracle():
    spp = 8
    want, _ = oracle_image(spp)
    s = build_product(spp)
    got = s.render(precision="f64", rng="chacha8").reshape(-1)
    assert got.shape == want.shape and np.all(np.isfinite(got))
    same = np.mean(got == want)
    rel = np.abs(got.astype(np.float64) - want) / np.maximum(np.abs(want.astype(np.float64)), 1e-30)
    assert same >= 0.999, f"bit-identical fraction {same:.5f}"
    assert np.max(rel) <= 1e-6, f"max rel err {np.max(rel):.3e}"
    # the motion matters: the same scene without speeds renders differently
    b = nrt.Builder()
    red, grey = b.solid((0.8, 0.2, 0.1)), b.solid((0.5, 0.5, 0.5))
    mats = [b.lambertian(red), b.metal(0.1, b.solid((0.8, 0.8, 0.9))), b.dielectric(1.5), b.lambertian(grey)]
    still = b.finish(b.bvh([b.sphere(c, r, mats[m]) for c, r, _, m in SPHERES]),
                     nrt.CameraBuilder(samples_per_pixel=spp, **CAM).build())
    assert np.mean(still.render(precision="f64", rng="chacha8").reshape(-1) != got) > 0.05


@pytest.mark.gpu
@pytest.mark.parametrize("precision,rng,trace", [("f32", "philox", "auto"), ("f32", "philox", "world-bvh"),
                                                 ("f32", "philox", "bvh"), ("f64", "philox", "auto")])
def test_moving_sphere_fast_variants_statistically_match(precision, rng, trace):
    spp = 64
    want, _, var = oracle_image(spp, var=True)
    want = want.astype(np.float64)
    var = np.maximum(var.astype(np.float64), 0.0)
    got = build_product(spp).render(precision=precision, rng=rng, trace=trace).reshape(-1).astype(np.float64)
    assert np.all(np.isfinite(got))
    for c in range(3):
        d = got[c::3].mean() - want[c::3].mean()
        se = np.sqrt(np.sum(2.0 * var[c::3] / spp)) / (W * H)
        assert abs(d) <= 4.5 * se + 1e-6, (c, d, se)
    k = 4

    def blocks(a):
        return a.reshape(H, W, 3).reshape(H // k, k, W // k, k, 3).mean(axis=(1, 3))

    vb = blocks(2.0 * var / spp) / (k * k)
    ok = vb > 1e-14
    z = (blocks(got) - blocks(want))[ok] / np.sqrt(vb[ok])
    med = float(np.median(np.abs(z)))
    assert 0.35 <= med <= 1.1, med
    assert np.mean(np.abs(z) > 5) < 0.03
