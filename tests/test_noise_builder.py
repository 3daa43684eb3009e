"""Perlin textures through the constructor API: nrt_texture_noise = PerlinRidgedNoiseBuilder
(lib/textures/noise.rs:30-101) and nrt_texture_marble = MarbleBuilder (lib/textures/marble.rs:24-60),
each builder field optional (an NRT_NOISE_* bit per Option) with the builders' defaults.  The scene
is built through the C ABI and, independently, as an oracle tree (oracle/oracle.cpp NoiseTex /
MarbleTex, the restated noise 0.9.0 Fbm<Perlin>: parity unpinned beyond the restatement).

CPU: the product's graph (texture parameters after the builders' defaults and Fbm's octave clamp)
equals the oracle's; bad field bits are refused.
GPU: the f64 / ChaCha8 kernel against the oracle (>= 99.9 % of values bit-identical, max relative
error 1e-6, as tests/test_gpu_parity.py), and the f32 / Philox world-mode kernel within the coarse
statistical screen of test_fast_variants_statistically_match.
"""
import math
import os
import tempfile

import numpy as np
import pytest

import nrt
from helpers import oracle_dump, oracle_render

W, H = 48, 32
CAM = dict(width=W, height=H, background_color=(0.7, 0.8, 1.0), look_from=(0.0, 1.2, 5.0), look_at=(0.0, 0.4, 0.0),
           view_up=(0.0, 1.0, 0.0), defocus_angle=0.0, focus_dist=1.0, field_of_view=0.8, ray_max_bounces=10)
LAC, PERS = math.pi * 2.0 / 3.0, 0.5  # Fbm::DEFAULT_LACUNARITY / DEFAULT_PERSISTENCE
# texture specs: (kind, builder kwargs, oracle tree fields after the defaults)
TEXTURES = [
    ("noise", dict(), (0, 1, 1.0, LAC, PERS)),                                    # every default
    ("noise", dict(seed=7, octaves=5, frequency=3.0, lacunarity=2.1, persistence=0.6), (7, 5, 3.0, 2.1, 0.6)),
    ("noise", dict(seed=3, octaves=0, frequency=8.0), (3, 1, 8.0, LAC, PERS)),     # set_octaves(0) clamps to 1
    ("noise", dict(octaves=99, persistence=0.4), (0, 32, 1.0, LAC, 0.4)),          # ... and 99 to 32
    ("marble", dict(), (0, 1.0)),
    ("marble", dict(seed=11, frequency=4.0), (11, 4.0)),
]


def _f(x):
    return float(x).hex()


def build_product(spp):
    b = nrt.Builder()
    tex = [getattr(b, kind)(**kw) for kind, kw, _ in TEXTURES]
    mats = [b.lambertian(t) for t in tex]
    light = b.diffuse_light(4.0, b.solid((1.0, 0.9, 0.8)))
    objs = [b.sphere((0.0, -1000.0, 0.0), 1000.0, mats[4]),
            b.sphere((-1.2, 0.5, 0.0), 0.5, mats[0]),
            b.sphere((0.0, 0.5, -0.4), 0.5, mats[1]),
            b.sphere((1.2, 0.5, 0.0), 0.5, mats[2]),
            b.quad((-2.0, 0.0, -1.5), (4.0, 0.0, 0.0), (0.0, 2.0, 0.0), mats[5]),
            b.triangle((-1.0, 0.05, 1.0), (0.8, 0.0, 0.0), (0.0, 0.6, 0.3), mats[3]),
            b.quad((-0.5, 2.5, -0.5), (1.0, 0.0, 0.0), (0.0, 0.0, 1.0), light)]
    cam = nrt.CameraBuilder(samples_per_pixel=spp, **CAM).build()
    return b.finish(b.bvh(objs), cam)


def oracle_tree_text(spp):
    c = CAM
    lines = [f"CAMERA {c['width']} {c['height']} {spp} {c['ray_max_bounces']} "
             + " ".join(_f(x) for x in (*c["background_color"], *c["look_from"], *c["look_at"], *c["view_up"]))
             + f" {_f(c['defocus_angle'])} {_f(c['focus_dist'])} {_f(c['field_of_view'])}"]
    for i, (kind, _, f) in enumerate(TEXTURES):
        if kind == "noise":
            lines.append(f"TEX {i} NOISE {f[0]} {f[1]} {_f(f[2])} {_f(f[3])} {_f(f[4])}")
        else:
            lines.append(f"TEX {i} MARBLE {f[0]} {_f(f[1])}")
    n = len(TEXTURES)
    lines.append(f"TEX {n} SOLID " + " ".join(_f(x) for x in (1.0, 0.9, 0.8)))
    lines += [f"MAT {i} LAMBERTIAN {i}" for i in range(n)] + [f"MAT {n} DIFFUSE_LIGHT {_f(4.0)} {n}"]
    sph = [((0.0, -1000.0, 0.0), 1000.0, 4), ((-1.2, 0.5, 0.0), 0.5, 0), ((0.0, 0.5, -0.4), 0.5, 1),
           ((1.2, 0.5, 0.0), 0.5, 2)]
    k = 0
    for ctr, r, m in sph:
        lines.append(f"OBJ {k} SPHERE " + " ".join(_f(x) for x in (*ctr, r)) + f" {m}")
        k += 1
    for kind, p, u, v, m in [("QUAD", (-2.0, 0.0, -1.5), (4.0, 0.0, 0.0), (0.0, 2.0, 0.0), 5),
                             ("TRIANGLE", (-1.0, 0.05, 1.0), (0.8, 0.0, 0.0), (0.0, 0.6, 0.3), 3),
                             ("QUAD", (-0.5, 2.5, -0.5), (1.0, 0.0, 0.0), (0.0, 0.0, 1.0), n)]:
        lines.append(f"OBJ {k} {kind} " + " ".join(_f(x) for x in (*p, *u, *v)) + f" {m}")
        k += 1
    lines += [f"OBJ {k} BVH {k} " + " ".join(str(i) for i in range(k)), f"ROOT {k}"]
    return "\n".join(lines) + "\n"


def oracle_image(spp, var=False):
    with tempfile.TemporaryDirectory() as td:
        tree = os.path.join(td, "noise.tree")
        with open(tree, "w") as fh:
            fh.write(oracle_tree_text(spp))
        return oracle_render(tree, var=var)


def _norm(text):
    out = []
    for line in text.splitlines()[1:]:  # the object graph (the camera lines are spelled differently)
        out.append(" ".join(repr(float.fromhex(t)) if t.startswith(("0x", "-0x")) else t for t in line.split()))
    return out


def test_noise_builder_graph_matches_oracle():
    got = "CAMERA\n" + build_product(4).dump()
    with tempfile.TemporaryDirectory() as td:
        tree = os.path.join(td, "noise.tree")
        with open(tree, "w") as fh:
            fh.write(oracle_tree_text(4))
        want = oracle_dump(tree)
    a, b = _norm(got), _norm(want)
    assert len(a) == len(b) and sum("NOISE" in x for x in a) == 4 and sum("MARBLE" in x for x in a) == 2
    for i, (x, y) in enumerate(zip(a, b)):
        assert x == y, f"line {i}:\nproduct {x}\noracle  {y}"


def test_noise_builder_defaults_equal_scene_file_defaults():
    # an empty `Noise {}` / `Marble {}` of a scene file and the builders with no field set are one texture
    b = nrt.Builder()
    d = b.finish(b.bvh([b.sphere((0, 0, 0), 1.0, b.lambertian(b.noise())),
                        b.sphere((0, 3, 0), 1.0, b.lambertian(b.marble()))])).dump()
    assert "NOISE 0 1" in d and "MARBLE 0 7" in d


def test_noise_builder_refuses_unknown_fields():
    b = nrt.Builder()
    L = nrt.lib()
    assert L.nrt_texture_noise(b._b, 1 << 5, 0, 0, 0.0, 0.0, 0.0) < 0
    assert "NRT_NOISE" in nrt.lib().nrt_last_error().decode()
    assert L.nrt_texture_marble(b._b, 2, 0, 0.0) < 0  # Marble has no octaves
    assert L.nrt_texture_marble(b._b, 5, 1, 2.0) >= 0


@pytest.mark.gpu
def test_noise_builder_f64_chacha8_matches_oracle():
    spp = 4
    want, _ = oracle_image(spp)
    got = build_product(spp).render(precision="f64", rng="chacha8").reshape(-1)
    assert got.shape == want.shape and np.all(np.isfinite(got))
    same = np.mean(got == want)
    rel = np.abs(got.astype(np.float64) - want) / np.maximum(np.abs(want.astype(np.float64)), 1e-30)
    assert same >= 0.999, f"bit-identical fraction {same:.5f}"
    assert np.max(rel) <= 1e-6, f"max rel err {np.max(rel):.3e}"


@pytest.mark.gpu
@pytest.mark.parametrize("trace", ["auto", "bvh"])
def test_noise_builder_f32_philox_statistically_matches(trace):
    spp = 64
    want, _, var = oracle_image(spp, var=True)
    want = want.astype(np.float64)
    var = np.maximum(var.astype(np.float64), 0.0)
    got = build_product(spp).render(precision="f32", rng="philox", trace=trace).reshape(-1).astype(np.float64)
    assert np.all(np.isfinite(got))
    for c in range(3):
        d = got[c::3].mean() - want[c::3].mean()
        se = np.sqrt(np.sum(2.0 * var[c::3] / spp)) / (W * H)
        assert abs(d) <= 4.5 * se + 1e-6, (c, d, se)
