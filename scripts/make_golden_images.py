"""Frozen oracle renders -> tests/golden/images/.

The oracle (test infrastructure: the C++ f64 restatement with the reference's
ChaCha8 stream) renders small frames of every BASELINE scene plus the other
loadable reference scenes; each frame is stored as little-endian f32 W x H x 3
(Rgb32FImage layout) next to manifest.json, which records the render parameters,
the sha256 of every input file the scene reads and of the frame itself.

    python scripts/make_golden_images.py
"""
import hashlib
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import helpers  # noqa: E402

# name -> (scene, W, H, spp, bounce cap or None)
CASES = {
    "cornell": ("scenes/cornell-box-scene.json", 48, 32, 4, None),
    "cornell_spp1": ("scenes/cornell-box-scene.json", 24, 16, 1, None),
    "cube": ("scenes/cube-scene.json", 40, 30, 4, None),
    "scale": ("scenes/scale.json", 32, 24, 4, None),
    "spheres": ("scenes/spheres.toml", 48, 27, 4, None),
    "quads": ("scenes/quads.toml", 32, 32, 4, None),
    "teapot": ("scenes/utah-teapot-scene.json", 32, 24, 2, None),
    "earth": ("scenes/earth.toml", 48, 27, 2, None),
    "triangles": ("scenes/triangles.toml", 40, 30, 4, None),
    "checker": ("scenes/checker.json", 48, 32, 4, None),
}
# files each scene reads (scene file, models it references, textures)
INPUTS = {
    "scenes/cornell-box-scene.json": ["scenes/cornell-box-model.json", "scenes/cube-model.toml"],
    "scenes/cube-scene.json": ["scenes/cube-model.toml"],
    "scenes/utah-teapot-scene.json": ["scenes/utah-teapot-model.toml"],
    "scenes/earth.toml": ["scenes/textures/earth.jpg", "scenes/textures/moon.jpg"],
}
OUT = os.path.join(ROOT, "tests", "golden", "images")


def sha256(path):
    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()


def render(scene, w, h, spp, bounces):
    with tempfile.TemporaryDirectory() as td:
        tree, _ = helpers.oracle_tree(scene, td, width=w, height=h, spp=spp, bounces=bounces)
        img, _ = helpers.oracle_render(tree, threads=os.cpu_count())
    return img


def main():
    helpers.ensure_oracle()
    os.makedirs(OUT, exist_ok=True)
    manifest = {"note": "oracle (f64, ChaCha8 reference stream) renders; little-endian f32 W x H x 3",
                "cases": {}}
    for name, (scene, w, h, spp, bounces) in CASES.items():
        img = render(scene, w, h, spp, bounces)
        path = os.path.join(OUT, name + ".f32")
        img.astype("<f4").tofile(path)
        files = [scene] + INPUTS.get(scene, [])
        manifest["cases"][name] = {
            "scene": scene, "width": w, "height": h, "spp": spp, "ray_max_bounces": bounces,
            "inputs": {f: sha256(os.path.join(helpers.GOLDEN, f)) for f in files},
            "image": name + ".f32", "image_sha256": sha256(path)}
        print(name, w, h, spp, manifest["cases"][name]["image_sha256"][:16], flush=True)
    with open(os.path.join(OUT, "manifest.json"), "w") as fh:
        json.dump(manifest, fh, indent=1)
        fh.write("\n")


if __name__ == "__main__":
    main()
