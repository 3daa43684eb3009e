"""ASan + UBSan run of the host stages (SURVEY §5 sanitizers row).

nr-ray-tracer_amd/build/san/host_check (make sanitize) is the JSON / TOML readers,
SceneConfig semantics, BVH build, flattener, f32 conversion and JPEG decoder built
with -fsanitize=address,undefined.  It runs over every reference scene and texture
plus malformed inputs made here with a fixed seed (truncations, byte mutations,
garbage, deep nesting).  Rejections are expected -- the library reports them as
status codes -- but no sanitizer report and no crash may occur.  Host code only:
GPU sanitizers are not available on this pool.
"""
import os
import random
import subprocess

import pytest

from helpers import GOLDEN, ROOT

PKG = os.path.join(ROOT, "nr-ray-tracer_amd")
BIN = os.path.join(PKG, "build", "san", "host_check")
SMALL = ["cornell-box-scene.json", "cornell-box-model.json", "cube-scene.json", "cube-model.toml", "scale.json",
         "quads.toml", "noise.toml", "simple-lights.toml", "earth.toml", "triangles.toml", "utah-teapot-scene.json"]


@pytest.fixture(scope="module")
def host_check():
    r = subprocess.run(["make", "-s", "-C", PKG, "sanitize"], capture_output=True, text=True)
    if r.returncode != 0 and ("asan" in r.stderr.lower() or "sanitize" in r.stderr.lower()):
        pytest.skip("no sanitizer runtime for g++ here: " + r.stderr[-300:])
    assert r.returncode == 0, r.stderr[-2000:]
    return BIN


def _run(binary, files):
    env = dict(os.environ, ASAN_OPTIONS="detect_leaks=0:abort_on_error=0:halt_on_error=1",
               UBSAN_OPTIONS="halt_on_error=1:print_stacktrace=1")
    r = subprocess.run([binary, "--quiet"] + files, capture_output=True, text=True, cwd=GOLDEN, env=env, timeout=600)
    report = r.stdout[-3000:] + r.stderr[-6000:]
    assert r.returncode == 0, report
    assert "AddressSanitizer" not in r.stderr and "runtime error" not in r.stderr, report
    return r.stdout


def test_reference_inputs_clean(host_check):
    files = sorted(os.path.join("scenes", f) for f in os.listdir(os.path.join(GOLDEN, "scenes")) if "." in f)
    files += ["scenes/textures/earth.jpg", "scenes/textures/moon.jpg"]
    out = _run(host_check, files)
    assert "loaded" in out


def test_malformed_inputs_clean(host_check, tmp_path):
    rnd = random.Random(20261016)
    files = []

    def put(name, data):
        p = tmp_path / name
        p.write_bytes(data)
        files.append(str(p))

    for f in SMALL:
        data = open(os.path.join(GOLDEN, "scenes", f), "rb").read()
        ext = os.path.splitext(f)[1]
        for k in range(12):  # truncations
            put(f"trunc{k}_{f}", data[: rnd.randrange(len(data))])
        for k in range(24):  # byte mutations (structural characters favoured)
            b = bytearray(data)
            for _ in range(rnd.randrange(1, 4)):
                i = rnd.randrange(len(b))
                b[i] = rnd.choice(b'[]{}",=:.-+e0123456789\n\x00\xff') if rnd.random() < 0.7 else rnd.randrange(256)
            put(f"mut{k}_{f}", bytes(b))
        put(f"empty{ext}", b"")
    for ext in (".json", ".toml"):
        put(f"garbage{ext}", bytes(rnd.randrange(256) for _ in range(4096)))
        put(f"deep{ext}", (b"a = " if ext == ".toml" else b"") + b"[" * 100000 + b"]" * 100000)
        put(f"bignum{ext}", (b"x = " if ext == ".toml" else b"") + b"1" * 5000)
    jpg = open(os.path.join(GOLDEN, "scenes", "textures", "moon.jpg"), "rb").read()
    for k in range(16):
        put(f"trunc{k}.jpg", jpg[: rnd.randrange(2, 4096) if k < 8 else rnd.randrange(len(jpg))])
    for k in range(32):
        b = bytearray(jpg)
        for _ in range(rnd.randrange(1, 6)):
            i = rnd.randrange(2, 2048) if k < 16 else rnd.randrange(2, len(b))  # headers, then entropy data
            b[i] = rnd.randrange(256)
        put(f"mut{k}.jpg", bytes(b))
    put("fill.jpg", b"\xff\xd8" + b"\xff" * 64)      # trailing fill bytes (jpeg.cpp marker loop)
    put("soi_only.jpg", b"\xff\xd8")
    out = _run(host_check, files)
    assert "rejected" in out
