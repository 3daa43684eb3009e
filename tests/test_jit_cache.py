"""On-disk cache of the scene-specialised kernels (csrc/jit.hip): a second process rendering the
same scene takes the code object from the cache instead of compiling it, renders the same bits, and
a damaged cache file is ignored (rebuilt), never loaded.  The reference has no counterpart (its
render is plain Rust); this serves the one-shot usage pattern of render.rs:57-62 (load, render
once, write the image), whose wall time the compile would otherwise dominate."""
import glob
import json
import os
import subprocess
import sys

import pytest

from helpers import ROOT

pytestmark = pytest.mark.gpu

CHILD = r"""
import hashlib, json, os, sys, time
sys.path.insert(0, os.path.join(sys.argv[1], "nr-ray-tracer_amd"))
import nrt
os.chdir(os.path.join(sys.argv[1], "tests", "golden"))
s = nrt.Scene.load("scenes/cornell-box-scene.json", nrt.CameraConfig(width=64, height=48, samples_per_pixel=8))
t0 = time.perf_counter()
img = s.render(precision="f32", rng="philox", device=0)
dt = time.perf_counter() - t0
print(json.dumps(dict(nrt.jit_stats(), sha=hashlib.sha256(img.tobytes()).hexdigest(), render_s=dt)))
"""


def _run(cache_dir):
    env = dict(os.environ, NRT_JIT_CACHE=str(cache_dir))
    env.pop("NRT_JIT", None)
    r = subprocess.run([sys.executable, "-c", CHILD, ROOT], capture_output=True, text=True, timeout=180, env=env)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    return json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])


def test_second_process_reads_the_disk_cache(tmp_path):
    first = _run(tmp_path)
    assert first["compiled"] == 1 and first["disk_hits"] == 0 and first["failed"] == 0
    files = glob.glob(str(tmp_path / "*.co"))
    assert len(files) == 1
    second = _run(tmp_path)
    assert second["compiled"] == 0 and second["disk_hits"] == 1 and second["launches"] >= 1
    assert second["sha"] == first["sha"]
    assert second["compile_s"] < 0.2  # a file read and a module load, no hiprtc


def test_damaged_cache_file_is_rebuilt(tmp_path):
    first = _run(tmp_path)
    (path,) = glob.glob(str(tmp_path / "*.co"))
    with open(path, "r+b") as fh:  # flip a byte inside the code object: the checksum no longer holds
        fh.seek(os.path.getsize(path) // 2)
        b = fh.read(1)
        fh.seek(-1, 1)
        fh.write(bytes([b[0] ^ 0xFF]))
    again = _run(tmp_path)
    assert again["disk_hits"] == 0 and again["compiled"] == 1
    assert again["sha"] == first["sha"]
    third = _run(tmp_path)  # the rebuilt file is whole again
    assert third["disk_hits"] == 1 and third["sha"] == first["sha"]


def test_untrusted_cache_directory_is_not_used(tmp_path):
    """A cache directory other users may write (here world-writable) could hand this process someone
    else's GPU code: the library neither reads nor writes it, and compiles in the process instead."""
    d = tmp_path / "shared"
    d.mkdir()
    os.chmod(d, 0o777)
    first = _run(d)
    assert first["compiled"] == 1 and first["disk_hits"] == 0 and first["failed"] == 0
    assert glob.glob(str(d / "*.co")) == []
    second = _run(d)
    assert second["compiled"] == 1 and second["disk_hits"] == 0 and second["sha"] == first["sha"]


def _fnv1a(data, h=1469598103934665603):
    for b in data:
        h = ((h ^ b) * 1099511628211) & 0xFFFFFFFFFFFFFFFF
    return h


def test_cache_file_the_runtime_refuses_is_replaced(tmp_path):
    """A cache file whose key and checksum hold but whose code object the HIP runtime refuses (another
    compiler's output, say) is deleted and compiled once more in the same process: the render uses the
    scene-specialised kernel, and the next process reads the rewritten file."""
    import struct
    first = _run(tmp_path)
    (path,) = glob.glob(str(tmp_path / "*.co"))
    buf = open(path, "rb").read()
    at = 8
    (klen,) = struct.unpack_from("<I", buf, at)
    at += 4 + klen
    (nlen,) = struct.unpack_from("<I", buf, at)
    at += 4 + nlen
    (clen,) = struct.unpack_from("<Q", buf, at)
    at += 8
    bad = bytearray(buf[:at]) + (b"not a code object " * (clen // 18 + 1))[:clen]
    bad += struct.pack("<Q", _fnv1a(bytes(bad)))
    open(path, "wb").write(bytes(bad))
    again = _run(tmp_path)
    assert again["disk_hits"] == 1 and again["compiled"] == 1 and again["failed"] == 0
    assert again["launches"] >= 1 and again["sha"] == first["sha"]
    third = _run(tmp_path)
    assert third["disk_hits"] == 1 and third["compiled"] == 0 and third["sha"] == first["sha"]
