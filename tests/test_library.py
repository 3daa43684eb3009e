"""libnrt.so: loads, exports every symbol include/nrt.h declares, and its host
logic behaves (no GPU compute here)."""
import ctypes
import math
import os
import re

import numpy as np
import pytest

import nrt
from helpers import ROOT

HEADER = os.path.join(ROOT, "include", "nrt.h")


def header_symbols():
    text = open(HEADER).read()
    text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
    return sorted(set(re.findall(r"\b(nrt_[a-z0-9_]+)\s*\(", text)))


def test_exports_every_declared_symbol():
    lib = ctypes.CDLL(nrt.LIB_PATH)
    syms = header_symbols()
    assert len(syms) >= 30
    missing = [s for s in syms if not hasattr(lib, s)]
    assert not missing, missing
    # the Python binding declares a signature for each of them
    assert sorted(nrt.SIGNATURES) == syms


def test_abi_version():
    assert nrt.lib().nrt_abi_version() == 7


def test_camera_builder_default_and_build():
    b = nrt.CameraBuilder()
    cam = b.build()
    # CameraBuilder::default (camera.rs:162-203) then build (94-159)
    assert (cam.width, cam.height, cam.samples_per_pixel, cam.ray_max_bounces) == (1200, 800, 10, 10)
    h = math.tan(math.pi / 2 / 2.0)
    vh = 1.0 * h * 2.0
    vw = vh * (1200 / 800)
    assert cam.pixel_delta_u[0] == pytest.approx(vw / 1200 / math.sqrt(2), rel=1e-12)
    assert cam.look_from == (1.0, 1.0, 1.0)
    b2 = nrt.CameraBuilder(samples_per_pixel=0).build()
    assert b2.samples_per_pixel == 1  # samples_per_pixel.max(1)


def test_camera_config_apply_degrees():
    b = nrt.CameraBuilder().apply(nrt.CameraConfig(field_of_view=35.0, defocus_angle=0.5, width=10, height=20))
    assert b.field_of_view == (35.0 * math.pi) / 180.0
    assert b.defocus_angle == (0.5 * math.pi) / 180.0
    assert (b.width, b.height) == (10, 20)


def test_to_rgb8_matches_image_crate_rules():
    x = np.array([0.0, 0.25, 1.0, 4.0, -1.0, np.nan, 0.5], dtype=np.float32)
    got = nrt.to_rgb8(x, 0.5)
    g = np.power(x, np.float32(0.5))
    want = []
    for v in g:
        c = 1.0 if not (v < 1.0) else max(v, 0.0)
        want.append(int(np.round(np.float32(c) * np.float32(255.0))))
    assert got.tolist() == want


def test_rows_selected():
    s = nrt.Builder()
    t = s.solid((0.5, 0.5, 0.5))
    m = s.lambertian(t)
    q = s.quad((0, 0, 0), (1, 0, 0), (0, 1, 0), m)
    scene = s.finish(s.bvh([q]))
    assert scene.rows_selected(1024, 0, 8) == 128
    assert scene.rows_selected(10, 3, 4) == 2   # rows 3, 7
    assert scene.rows_selected(10, 10, 4) == 0
    assert scene.rows_selected(7, 0, 1) == 7


def test_builder_errors_are_reported_not_fatal():
    b = nrt.Builder()
    with pytest.raises(nrt.NrtError) as ei:
        b.lambertian(5)
    assert ei.value.code == -1 and "texture handle" in str(ei.value)
    t = b.solid((1, 1, 1))
    m = b.lambertian(t)
    sph = b.sphere((0, 0, 0), 1.0, m)
    with pytest.raises(nrt.NrtError):
        b.finish(sph)  # root must be a BVH


def test_builder_matches_loader_dump():
    # The constructor API builds the same graph as a scene file does.
    b = nrt.Builder()
    t = b.solid((0.5, 0.5, 0.5))
    m = b.lambertian(t)
    q = [b.quad((0, 0, 0), (1, 0, 0), (0, 1, 0), m), b.quad((0, 0, 1), (1, 0, 0), (0, 1, 0), m),
         b.quad((0, 1, 0), (1, 0, 0), (0, 0, 1), m)]
    inner = b.bvh(q)
    obj = b.translate(b.rotate("y", b.scale(inner, (0.5, 2.0, 1.0)), 0.3), (1.0, 0.0, -1.0))
    scene = b.finish(b.bvh([obj, b.sphere((0, 2, 0), 0.5, m)]))
    d = scene.dump()
    assert d.count("QUAD") == 3 and "SCALE" in d and "ROTATE" in d and "TRANSLATE" in d
    st = scene.stats()
    assert st["instances"] == 1 and st["xforms"] == 3 and st["prims"] == 4


def test_render_without_gpu_fails_loudly():
    if nrt.device_count() > 0:
        pytest.skip("a GPU is visible")
    b = nrt.Builder()
    m = b.lambertian(b.solid((1, 1, 1)))
    scene = b.finish(b.bvh([b.sphere((0, 0, 0), 1.0, m)]))
    cam = nrt.CameraBuilder(width=4, height=4, samples_per_pixel=1).build()
    with pytest.raises(nrt.NrtError) as ei:
        scene.render(cam)
    assert ei.value.code == -3


@pytest.mark.parametrize("scene,pairs,list_ok", [
    ("scenes/cornell-box-scene.json", 2, 1),   # both cubes stand on the floor (y = 0)
    ("scenes/scale.json", 1, 1),
    ("scenes/cube-scene.json", 2, 0),          # touching cube faces: world BVH keys, not the list
    ("scenes/utah-teapot-scene.json", 0, 1),
    ("scenes/spheres.toml", 0, 1),
])
def test_coplanar_ties_detected(scene, pairs, list_ok):
    """Overlapping coplanar surfaces tie exactly in the reference (BVH::hit picks the later
    candidate, object.rs:109-115); the flattener finds them and keeps the world list only
    where its f32 formulas tie bit for bit (device_scene.hpp WCLASS_*)."""
    from helpers import in_golden

    with in_golden():
        s = nrt.Scene.load(scene, nrt.CameraConfig(width=8, height=8, samples_per_pixel=1))
    st = s.stats()
    assert st["coplanar_pairs"] == pairs
    assert st["world_list_ok"] == list_ok


@pytest.mark.parametrize("scene,mode", [
    ("scenes/cornell-box-scene.json", 2),   # world-BVH culling wherever the slots map
    ("scenes/scale.json", 2),
    ("scenes/utah-teapot-scene.json", 2),   # 7520 triangles under one instance: world-BVH culling
    ("scenes/spheres.toml", 2),             # 488 spheres, no instances
])
def test_exact_mode(scene, mode):
    """The reference-exact kernel's traversal (nrt.h nrt_exact_mode): the f32 world BVH culls,
    each of its slots mapped onto the reference primitive and instance it came from; small
    scenes without that mapping test every primitive in depth-first order."""
    from helpers import in_golden

    with in_golden():
        s = nrt.Scene.load(scene, nrt.CameraConfig(width=8, height=8, samples_per_pixel=1))
    assert s.stats()["exact_mode"] == mode


@pytest.mark.parametrize("n,mode", [(60, 0), (10, 1)])
def test_exact_mode_nested_instances(n, mode):
    """Nested instances have no single object-space ray per primitive: no world-BVH mapping, so
    the exact kernel walks every primitive (small scenes, NRT_EXACT_ALL) or keeps the reference
    tree (NRT_EXACT_BVH)."""
    b = nrt.Builder()
    m = b.lambertian(b.solid((0.5, 0.5, 0.5)))
    quads = [b.quad((i, 0, 0), (0.5, 0, 0), (0, 0.5, 0), m) for i in range(n)]
    inner = b.translate(b.bvh(quads), (0.0, 1.0, 0.0))
    outer = b.rotate("y", b.bvh([inner]), 0.25)
    s = b.finish(b.bvh([outer]))
    assert s.stats()["exact_mode"] == mode


def test_library_built_from_these_sources():
    """Build provenance: the loaded libnrt.so carries the hash of the sources it was
    compiled from; it must equal the hash of csrc/ + include/nrt.h in this tree."""
    assert nrt.build_id() == nrt.source_hash()


@pytest.mark.parametrize("targs", [
    # Cornell's world list (ABOX x1, QUAD_Y x1, BOXY x2), KF_FLAT, scene staged in LDS
    "float, nrt::dev::Philox, 0, false, true, 4, nrt::dev::WorldSig<23u, 21u, 40u>",
    # the teapot's world BVH (4-wide, no coplanar ties), KF_FLAT, unstaged
    "float, nrt::dev::Philox, -1, false, false, 4, nrt::dev::BvhSig<4, false>",
    # the same two with the reference's ChaCha8 stream (one lane per pixel)
    "float, nrt::dev::ChaCha8, 0, false, true, 4, nrt::dev::WorldSig<23u, 21u, 40u>",
    "float, nrt::dev::ChaCha8, -1, false, false, 4, nrt::dev::BvhSig<4, false>",
    # the teapot's compact tree (16-bit refs, triangles only: LDS node cache), a world list with
    # an f64 and an f32 sphere run (a sphere anchored outside the scene scale beside one inside),
    # and the earth's world list (one f32 sphere run; not KF_FLAT)
    "float, nrt::dev::Philox, -1, false, false, 4, nrt::dev::BvhSig<5, false, 2>",
    "float, nrt::dev::Philox, 0, false, true, 0, nrt::dev::WorldSig<16u, 41u>",
    "float, nrt::dev::Philox, 0, false, true, 0, nrt::dev::WorldSig<57u>",
])
def test_scene_specialised_kernel_compiles(targs):
    """The device headers embedded in libnrt.so still compile under hiprtc (jit.hip), so a GPU
    run builds the scene-specialised kernels instead of falling back to the generic ones."""
    assert nrt.debug_jit_compile(targs) > 4096
    with pytest.raises(nrt.NrtError):
        nrt.debug_jit_compile("float, nrt::dev::NoSuchRng, 0")


def test_render_argument_errors_are_invalid():
    """Bad render arguments are NRT_E_INVALID (-1) whether or not a GPU is present (checked before any
    device work): gpus >= 1 renders the whole frame, so a row subset with it is refused."""
    b = nrt.Builder()
    m = b.lambertian(b.solid((1, 1, 1)))
    scene = b.finish(b.bvh([b.sphere((0, 0, 0), 1.0, m)]))
    cam = nrt.CameraBuilder(width=4, height=4, samples_per_pixel=1).build()
    with pytest.raises(nrt.NrtError) as ei:
        scene.render(cam, gpus=1, row_offset=1, row_stride=2)
    assert ei.value.code == -1 and "whole frame" in str(ei.value)
    with pytest.raises(nrt.NrtError) as ei:
        scene.render(cam, precision="f32", rng="philox", device=10 ** 6)
    assert ei.value.code in (-1, -3)  # device ordinal out of range (-1), or no GPU at all (-3)


def test_chacha8_probe_streams_below_2_32():
    """ChaCha8 streams are pixel indices, below 2^32 (images are capped below 2^32 pixels, and the
    kernels fold the stream's zero high word): the probe refuses streams past that before any device
    work, whether or not a GPU is present."""
    with pytest.raises(nrt.NrtError) as ei:
        nrt.debug_rng("chacha8", 2 ** 32 - 8, 64, 4)
    assert ei.value.code == -1 and "2^32" in str(ei.value)


def test_bench_refuses_multi_gpu_loopback():
    """NRT_MULTI_LOOPBACK (the library's test-only N-shards-on-one-GPU mode) never produces a bench line."""
    import subprocess
    import sys
    env = dict(os.environ, NRT_MULTI_LOOPBACK="1")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], capture_output=True, text=True,
                       env=env, timeout=60)
    assert r.returncode != 0 and "NRT_MULTI_LOOPBACK" in r.stderr
    assert not [l for l in r.stdout.splitlines() if l.startswith("{")]


def test_render_prepare_without_gpu_is_a_device_error():
    """nrt_render_prepare (ABI 7) reports a missing GPU as NRT_E_DEVICE, like the render calls."""
    if nrt.device_count() > 0:
        pytest.skip("a GPU is visible")
    b = nrt.Builder()
    m = b.lambertian(b.solid((0.5, 0.5, 0.5)))
    s = b.finish(b.bvh([b.sphere((0, 0, 0), 0.5, m)]), nrt.CameraBuilder(width=4, height=4).build())
    with pytest.raises(nrt.NrtError) as e:
        s.prepare(gpus=2)
    assert e.value.code == -3
