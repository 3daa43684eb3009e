"""Reference-exact fixtures at the BASELINE configurations' sizes -> tests/golden/baseline/.

The reference's per-pixel stream runs across ALL spp samples of a pixel (camera.rs:318-331: one
ChaCha8Rng per pixel, `set_stream(pixel index)`, then spp samples drawn from it in order), so at
spp 256 a pixel's last samples sit ~1 600 ChaCha8 blocks into a stream, and pixel indices reach
2^20 (1024 x 1024) or 2^21 (1920 x 1080).  The small parity cases (tests/test_gpu_parity.py) stop
at 64 x 40 and spp 8.  These fixtures are the oracle (test infrastructure: the C++ f64 restatement
of the reference path, oracle/oracle.cpp) rendering each BASELINE.json configuration at its full
image size and spp, over a row sample (rows y = (H - 1) mod stride (mod stride), so the frame's
last row, with the largest pixel indices, is in it: every pixel index of those rows is the one the
full frame uses), stored as little-endian f32 rows x W x 3 (Rgb32FImage rows).
tests/test_baseline_parity.py renders the same rows with the f64 / ChaCha8 kernel (nrt_render_opts
row_offset, row_stride) and requires >= 99.9 % bit-identical values, max relative error <= 1e-6.

    python scripts/make_baseline_fixtures.py [name ...]      (~1-2 minutes on 8 cores)
"""
import hashlib
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import helpers  # noqa: E402

# name -> (BASELINE.json config, scene, W, H, spp, row stride)
CASES = {
    "c1_spheres": ("configs[0]", "scenes/spheres.toml", 400, 225, 16, 1),
    "c2_cornell": ("configs[1]", "scenes/cornell-box-scene.json", 512, 512, 64, 16),
    "c3_earth": ("configs[2]", "scenes/earth.toml", 1920, 1080, 128, 216),
    "c4_teapot": ("configs[3]", "scenes/utah-teapot-scene.json", 1024, 1024, 256, 64),
    "c5_cornell": ("configs[4]", "scenes/cornell-box-scene.json", 1024, 1024, 256, 64),
}
INPUTS = {
    "scenes/cornell-box-scene.json": ["scenes/cornell-box-model.json", "scenes/cube-model.toml"],
    "scenes/utah-teapot-scene.json": ["scenes/utah-teapot-model.toml"],
    "scenes/earth.toml": ["scenes/textures/earth.jpg", "scenes/textures/moon.jpg"],
}
OUT = os.path.join(ROOT, "tests", "golden", "baseline")


def sha256(path):
    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()


def render(name):
    """The oracle's rows of case `name` (f32 array, rows x W x 3 flattened) and its stats."""
    _, scene, w, h, spp, stride = CASES[name]
    with tempfile.TemporaryDirectory() as td:
        tree, _ = helpers.oracle_tree(scene, td, width=w, height=h, spp=spp)
        return helpers.oracle_render(tree, threads=os.cpu_count(), rows=(row_offset(name), stride))


def row_offset(name):
    """The sample's first row: the frame's last row is in the sample."""
    _, _, _, h, _, stride = CASES[name]
    return (h - 1) % stride


def main(names):
    helpers.ensure_oracle()
    os.makedirs(OUT, exist_ok=True)
    mpath = os.path.join(OUT, "manifest.json")
    manifest = {"note": "oracle (f64, ChaCha8 reference stream) renders of the BASELINE.json configurations at "
                        "full size and spp over rows y = row_offset (mod row_stride); little-endian f32 rows x W x 3; made "
                        "by scripts/make_baseline_fixtures.py",
                "cases": {}}
    if os.path.exists(mpath):
        with open(mpath) as fh:
            manifest["cases"].update(json.load(fh).get("cases", {}))
    for name in names or list(CASES):
        config, scene, w, h, spp, stride = CASES[name]
        t0 = time.time()
        img, info = render(name)
        off = row_offset(name)
        rows = (h - off + stride - 1) // stride
        assert img.size == rows * w * 3, (img.size, rows, w)
        path = os.path.join(OUT, name + ".f32")
        img.astype("<f4").tofile(path)
        files = [scene] + INPUTS.get(scene, [])
        manifest["cases"][name] = {
            "baseline": config, "scene": scene, "width": w, "height": h, "spp": spp, "row_offset": off,
            "row_stride": stride, "rows": rows, "max_pixel_index": (off + (rows - 1) * stride) * w + w - 1,
            "inputs": {f: sha256(os.path.join(helpers.GOLDEN, f)) for f in files},
            "image": name + ".f32", "image_sha256": sha256(path),
            "oracle_seconds": round(time.time() - t0, 1), "oracle_threads": info.get("threads"),
            "samples": info.get("samples")}
        print(name, w, h, spp, f"rows {rows}", f"{time.time() - t0:.1f}s", flush=True)
    with open(mpath, "w") as fh:
        json.dump(manifest, fh, indent=1)
        fh.write("\n")


if __name__ == "__main__":
    main(sys.argv[1:])
