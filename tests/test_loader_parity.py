"""Product loader + BVH builder (C++, libnrt.so) vs the oracle's independent build.

Both sides restate scene_config.rs / cli.rs / object.rs; the canonical dump
(hex floats for every bbox, transform matrix, primitive precompute, material and
camera field) must be identical, which pins the flattener's input bit-for-bit.
CPU only: no render is performed.
"""
import os
import tempfile

import pytest

import nrt
from helpers import in_golden, is_legacy, oracle_dump, oracle_tree

# (scene, overrides) — every scene file in the reference that its own loader accepts
LOADABLE = [
    ("scenes/cornell-box-scene.json", dict(width=64, height=48, spp=16)),
    ("scenes/cornell-box-scene.json", dict()),
    ("scenes/cube-scene.json", dict(width=40, height=30, spp=2)),
    ("scenes/scale.json", dict(width=33, height=17, spp=1)),
    ("scenes/spheres.toml", dict(width=400, height=225, spp=16)),
    ("scenes/quads.toml", dict()),
    ("scenes/cornell-box-model.json", dict(width=8, height=8)),
    ("scenes/cube-model.toml", dict(width=8, height=8)),
    ("scenes/utah-teapot-scene.json", dict(width=64, height=64, spp=4)),  # generated model (Q16)
    ("scenes/earth.toml", dict(width=64, height=36, spp=2)),              # two 2048x1024 JPEG textures
    ("scenes/noise.toml", dict(width=40, height=30, spp=2)),              # Perlin Noise + Marble textures
    ("scenes/simple-lights.toml", dict(width=40, height=30, spp=2)),      # Marble + lights
    ("scenes/triangles.toml", dict(width=40, height=30, spp=2)),          # legacy index schema (Q14)
    ("scenes/checker.json", dict(width=40, height=30, spp=2)),            # Checker textures (test scene)
]


def product_dump(scene, ov):
    cfg = nrt.CameraConfig(width=ov.get("width"), height=ov.get("height"), samples_per_pixel=ov.get("spp"),
                           ray_max_bounces=ov.get("bounces"))
    with in_golden():
        s = nrt.Scene.load(scene, cfg, legacy_schema=is_legacy(scene))
    c = s.camera

    def hx3(v):
        return "".join(" " + float(x).hex().replace("0x0.0p+0", "0x0p+0") for x in v)

    cam = (f"CAMERA {c.width} {c.height} {c.samples_per_pixel} {c.ray_max_bounces}" + hx3(c.background_color)
           + hx3(c.look_from) + hx3(c.defocus_disk_u) + hx3(c.defocus_disk_v) + hx3(c.pixel_delta_u)
           + hx3(c.pixel_delta_v) + hx3(c.top_left) + "\n")
    return cam + s.dump(), s


def _norm(text):
    # printf("%a") and float.hex() spell a few values differently; compare numerically per token
    out = []
    for line in text.splitlines():
        toks = []
        for t in line.split():
            if t.startswith(("0x", "-0x")) or t in ("inf", "-inf", "nan", "-nan"):
                v = float.fromhex(t) if "0x" in t else float(t)
                toks.append("nan" if v != v else repr(v))
            else:
                toks.append(t)
        out.append(" ".join(toks))
    return out


@pytest.mark.parametrize("scene,ov", LOADABLE, ids=[f"{s}-{i}" for i, (s, _) in enumerate(LOADABLE)])
def test_dump_matches_oracle(scene, ov):
    with tempfile.TemporaryDirectory() as td:
        tree, _ = oracle_tree(scene, td, width=ov.get("width"), height=ov.get("height"), spp=ov.get("spp"),
                              bounces=ov.get("bounces"))
        want = oracle_dump(tree)
    got, _ = product_dump(scene, ov)
    a, b = _norm(got), _norm(want)
    assert len(a) == len(b)
    for i, (x, y) in enumerate(zip(a, b)):
        assert x == y, f"line {i}:\nproduct {x}\noracle  {y}"


def test_cornell_flat_counts():
    # 18 quads, 17 inner nodes, 2 instance chains of depth 4
    _, s = product_dump("scenes/cornell-box-scene.json", {})
    st = s.stats()
    assert st["prims"] == 18
    assert st["instances"] == 2
    assert st["xforms"] == 8
    assert st["max_instance_depth"] == 1
    assert st["nodes"] == 17 + 18 + 2
    assert st["trees"] == 3


def test_spheres_counts():
    _, s = product_dump("scenes/spheres.toml", dict(width=40, height=20))
    st = s.stats()
    assert st["prims"] == 488
    assert st["nodes"] == 488 + 487
    assert st["instances"] == 0


# `nr-ray-tracer create triangles` (create/triangles.rs:10-117) in the current schema: the same
# scene as the legacy scenes/triangles.toml, with named ids instead of indices (and the file's
# +0.0 where today's 4.0 * DVec3::NEG_Z would write -0.0)
TRIANGLES_CURRENT = """{
 "camera": {"background_color": [0.7, 0.8, 1.0], "look_from": [0.0, 0.0, 9.0], "look_at": [0.0, 0.0, 0.0],
            "field_of_view": 80.0, "ray_max_bounces": 10, "samples_per_pixel": 10},
 "textures": [["solid_red", {"SolidColor": {"color": [1.0, 0.2, 0.2]}}],
              ["solid_green", {"SolidColor": {"color": [0.2, 1.0, 0.2]}}],
              ["solid_blue", {"SolidColor": {"color": [0.2, 0.2, 1.0]}}],
              ["solid_orange", {"SolidColor": {"color": [1.0, 0.5, 0.0]}}],
              ["solid_cyan", {"SolidColor": {"color": [0.2, 0.8, 0.8]}}]],
 "materials": [["lambertian_red", {"Lambertian": {"texture": "solid_red"}}],
               ["lambertian_green", {"Lambertian": {"texture": "solid_green"}}],
               ["lambertian_blue", {"Lambertian": {"texture": "solid_blue"}}],
               ["lambertian_orange", {"Lambertian": {"texture": "solid_orange"}}],
               ["lambertian_cyan", {"Lambertian": {"texture": "solid_cyan"}}]],
 "scene": [
  {"Triangle": {"point": [-3.0, -2.0, 5.0], "u": [0.0, 0.0, -4.0], "v": [0.0, 4.0, 0.0], "material": "lambertian_red"}},
  {"Triangle": {"point": [-2.0, -2.0, 0.0], "u": [4.0, 0.0, 0.0], "v": [0.0, 4.0, 0.0], "material": "lambertian_green"}},
  {"Triangle": {"point": [3.0, -2.0, 1.0], "u": [0.0, 0.0, 4.0], "v": [0.0, 4.0, 0.0], "material": "lambertian_blue"}},
  {"Triangle": {"point": [-2.0, 3.0, 1.0], "u": [4.0, 0.0, 0.0], "v": [0.0, 0.0, 4.0], "material": "lambertian_orange"}},
  {"Triangle": {"point": [-2.0, -3.0, 5.0], "u": [4.0, 0.0, 0.0], "v": [0.0, 0.0, -4.0], "material": "lambertian_cyan"}}
 ]
}"""


def test_legacy_triangles_equal_current_schema(tmp_path):
    """scenes/triangles.toml (index-based legacy schema, triangles.toml:22-189) loads as the scene
    today's `create triangles` writes (create/triangles.rs): identical canonical dumps."""
    cur = tmp_path / "triangles-current.json"
    cur.write_text(TRIANGLES_CURRENT)
    ov = dict(width=40, height=30, spp=2)
    legacy, _ = product_dump("scenes/triangles.toml", ov)
    current, _ = product_dump(str(cur), ov)
    assert _norm(legacy) == _norm(current)
    with tempfile.TemporaryDirectory() as td:  # and the oracle's independent loader agrees
        tree, _ = oracle_tree(str(cur), td, width=40, height=30, spp=2)
        assert _norm(oracle_dump(tree)) == _norm(current)


@pytest.mark.parametrize("scene,code", [
    ("scenes/does-not-exist.json", -2),
    ("scenes/textures/earth.jpg", -2),       # not a scene format
    ("scenes/triangles.toml", -2),           # legacy index schema: rejected by default, as by the reference
])
def test_load_errors(scene, code):
    with in_golden():
        with pytest.raises(nrt.NrtError) as ei:
            nrt.Scene.load(scene)
    assert ei.value.code == code


def test_size_rules():
    # cli.rs:273-312: W alone is an error; W + ratio derives H; all three conflict
    with in_golden():
        with pytest.raises(nrt.NrtError):
            nrt.Scene.load("scenes/cornell-box-scene.json", nrt.CameraConfig(width=10))
        s = nrt.Scene.load("scenes/cornell-box-scene.json", nrt.CameraConfig(width=100, aspect_ratio=16 / 9))
        assert (s.camera.width, s.camera.height) == (100, 56)
        s = nrt.Scene.load("scenes/cornell-box-scene.json", nrt.CameraConfig(height=90, aspect_ratio=16 / 9))
        assert (s.camera.width, s.camera.height) == (160, 90)
        with pytest.raises(nrt.NrtError):
            nrt.Scene.load("scenes/cornell-box-scene.json", nrt.CameraConfig(width=1, height=1, aspect_ratio=1.0))
        s = nrt.Scene.load("scenes/cornell-box-scene.json")
        assert (s.camera.width, s.camera.height) == (1200, 800)  # CameraBuilder default
        assert s.camera.samples_per_pixel == 200 and s.camera.ray_max_bounces == 50


def test_legacy_schema_is_opt_in(tmp_path):
    """The reference's SceneConfig (scene_config.rs:384-404) expects (id, config) pairs and ignores
    an unknown `objects` key: scenes/triangles.toml fails to load and a current-schema document with
    `objects` but no `scene` loads as an empty scene, unless the legacy schema is asked for
    (nrt_scene_load_ex NRT_LOAD_LEGACY_SCHEMA); the oracle's loader agrees on both."""
    from oracle import scene_tree

    with in_golden():
        with pytest.raises(scene_tree.LoadError):
            scene_tree.load_doc("scenes/triangles.toml") and scene_tree.build_tree(
                "scenes/triangles.toml", None, str(tmp_path))
        s = nrt.Scene.load("scenes/triangles.toml", nrt.CameraConfig(width=8, height=8), legacy_schema=True)
        assert s.stats()["prims"] > 0
    doc = tmp_path / "objects-only.json"
    doc.write_text('{"camera": {}, "objects": [{"Sphere": {"center": [0, 0, 0], "radius": 1.0}}]}')
    empty = nrt.Scene.load(str(doc), nrt.CameraConfig(width=8, height=8))
    assert empty.stats()["prims"] == 0
    assert nrt.Scene.load(str(doc), nrt.CameraConfig(width=8, height=8), legacy_schema=True).stats()["prims"] == 1
