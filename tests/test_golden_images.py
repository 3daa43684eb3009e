"""Frozen oracle renders (tests/golden/images, written by scripts/make_golden_images.py).

CPU: the committed inputs are the ones the fixtures were made from (sha256), and the
oracle still reproduces every fixture bit for bit.  GPU: the reference-exact kernel
(f64, ChaCha8 stream) against the fixtures with the bar of test_gpu_parity.py
(>= 99.9 % of floats bit-identical, max relative error <= 1e-6), so the HIP path is
checked against stored reference-path outputs without running the oracle.
"""
import hashlib
import json
import os
import tempfile

import numpy as np
import pytest

from helpers import is_legacy, GOLDEN, in_golden, oracle_render, oracle_tree

IMAGES = os.path.join(GOLDEN, "images")
with open(os.path.join(IMAGES, "manifest.json")) as _fh:
    MANIFEST = json.load(_fh)["cases"]


def _fixture(name):
    c = MANIFEST[name]
    img = np.fromfile(os.path.join(IMAGES, c["image"]), dtype="<f4")
    assert img.size == c["width"] * c["height"] * 3
    return c, img


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_inputs_and_fixture_hashes(name):
    c = MANIFEST[name]
    for f, digest in c["inputs"].items():
        with open(os.path.join(GOLDEN, f), "rb") as fh:
            assert hashlib.sha256(fh.read()).hexdigest() == digest, f
    with open(os.path.join(IMAGES, c["image"]), "rb") as fh:
        assert hashlib.sha256(fh.read()).hexdigest() == c["image_sha256"]


@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_oracle_reproduces_fixture(name):
    c, want = _fixture(name)
    with tempfile.TemporaryDirectory() as td:
        tree, _ = oracle_tree(c["scene"], td, width=c["width"], height=c["height"], spp=c["spp"],
                              bounces=c["ray_max_bounces"])
        got, _ = oracle_render(tree, threads=4)
    np.testing.assert_array_equal(got, want)


@pytest.mark.gpu
@pytest.mark.parametrize("name", sorted(MANIFEST))
def test_exact_kernel_matches_fixture(name):
    import nrt

    c, want = _fixture(name)
    with in_golden():
        s = nrt.Scene.load(c["scene"], nrt.CameraConfig(width=c["width"], height=c["height"],
                                                        samples_per_pixel=c["spp"],
                                                        ray_max_bounces=c["ray_max_bounces"]),
                           legacy_schema=is_legacy(c["scene"]))
    got = s.render(precision="f64", rng="chacha8").reshape(-1)
    assert np.all(np.isfinite(got))
    same = np.mean(got == want)
    rel = np.abs(got.astype(np.float64) - want) / np.maximum(np.abs(want.astype(np.float64)), 1e-30)
    assert same >= 0.999, f"bit-identical fraction {same:.5f}"
    assert np.max(rel) <= 1e-6, f"max rel err {np.max(rel):.3e}"
