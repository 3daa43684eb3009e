"""Known-answer geometry test, independent of the oracle's code.

With spp = 1 the camera does not jitter (camera.rs:250-254) and without a defocus
angle every primary ray starts at look_from, so the primary ray of pixel (x, y) is
closed-form (CameraBuilder::build camera.rs:94-159, get_ray camera.rs:244-267).
With ray_max_bounces = 1 a pixel of the Cornell box is the light's emission when the
primary ray's nearest hit is the light quad (DiffuseLight::emit on a ray whose bounce
flag is 0 gives 1 x the white texture, diffuse_light.rs:62-75; Q4), and black
otherwise: a scattered ray meets the depth cap (Q6), a miss sees the black background.
The expected image is computed here in numpy from the scene file's numbers (the light
sits 0.002 below the ceiling and above both blocks, so no other surface comes first),
with the quad's closed [0, 1]^2 test of plane.rs:121-126.  Pixels whose planar
coordinates lie within 1e-9 of the quad's border are excluded (ulp-level ties; 1e-4
for the f32 kernels, whose camera rays are f32).
"""
import json
import os
import tempfile

import numpy as np
import pytest

from helpers import SCENES, oracle_render, oracle_tree

W = H = 96
SCENE = "scenes/cornell-box-scene.json"


def expected_mask(border=1e-9):
    with open(os.path.join(SCENES, "cornell-box-scene.json")) as fh:
        cam = json.load(fh)["camera"]
    with open(os.path.join(SCENES, "cornell-box-model.json")) as fh:
        light = [o["Quad"] for o in json.load(fh)["scene"] if o["Quad"]["material"] == "mat_0000003"][0]
    look_from, look_at = np.array(cam["look_from"], float), np.array(cam["look_at"], float)
    fov = cam["field_of_view"] * np.pi / 180.0   # cli.rs:369-371
    focus = 1.0                                   # DEFAULT_FOCUS_DISTANCE (camera.rs:175)
    up = np.array([0.0, 1.0, 0.0])                # DEFAULT_VIEW_UP
    vh = focus * np.tan(fov / 2) * 2.0
    vw = vh * (W / H)
    w = (look_from - look_at) / np.linalg.norm(look_from - look_at)
    u = np.cross(up, w); u /= np.linalg.norm(u)
    v = np.cross(w, u); v /= np.linalg.norm(v)
    vu, vv = u * vw, -v * vh
    du, dv = vu / W, vv / H
    top_left = look_from - w * focus - vu / 2 - vv / 2 + (du + dv) / 2
    ys, xs = np.mgrid[0:H, 0:W]
    d = top_left + xs[..., None] * du + ys[..., None] * dv - look_from  # (H, W, 3)
    q, qu, qv = (np.array(light[k], float) for k in ("point", "u", "v"))
    n = np.cross(qu, qv)
    nn = n / np.linalg.norm(n)
    wq = n / n.dot(n)
    denom = d @ nn
    t = (nn.dot(q) - nn.dot(look_from)) / denom
    p = look_from + t[..., None] * d - q
    alpha = np.cross(p, qv) @ wq
    beta = np.cross(qu, p) @ wq
    hit = (np.abs(denom) >= 1e-8) & (t > 0.001) & (alpha >= 0) & (alpha <= 1) & (beta >= 0) & (beta <= 1)
    edge = np.minimum.reduce([np.abs(alpha), np.abs(alpha - 1), np.abs(beta), np.abs(beta - 1)]) < border
    return hit, edge


def _camera_config():
    import nrt
    return nrt.CameraConfig(width=W, height=H, samples_per_pixel=1, ray_max_bounces=1)


def test_expected_mask_is_nontrivial():
    hit, edge = expected_mask()
    assert 30 < hit.sum() < hit.size // 50  # the light, seen almost edge-on near the top of the frame
    assert hit[: H // 3].sum() == hit.sum()
    assert edge.sum() == 0


def test_oracle_matches_closed_form():
    hit, edge = expected_mask()
    with tempfile.TemporaryDirectory() as td:
        tree, _ = oracle_tree(SCENE, td, width=W, height=H, spp=1, bounces=1)
        img, _ = oracle_render(tree, threads=4)
    img = img.reshape(H, W, 3)
    want = np.where(hit[..., None], 1.0, 0.0).astype(np.float32)
    keep = ~edge
    assert np.array_equal(img[keep], np.broadcast_to(want, img.shape)[keep])


@pytest.mark.gpu
@pytest.mark.parametrize("precision,rng", [("f64", "chacha8"), ("f32", "chacha8"), ("f32", "philox"),
                                           ("f64", "philox")])
def test_kernel_matches_closed_form(precision, rng):
    import nrt
    from helpers import in_golden

    hit, edge = expected_mask(1e-9 if precision == "f64" else 1e-4)
    assert edge.sum() <= 4
    with in_golden():
        scene = nrt.Scene.load(SCENE, _camera_config())
    img = scene.render(precision=precision, rng=rng)
    want = np.where(hit[..., None], 1.0, 0.0).astype(np.float32)
    keep = ~edge
    assert np.array_equal(img[keep], np.broadcast_to(want, img.shape)[keep])
