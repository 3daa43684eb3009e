"""High-sample oracle fixtures for the statistical tolerance of SURVEY §8(d) -> tests/golden/stat/.

The fast kernels (f32 and/or Philox) draw different random numbers from the
reference's per-pixel ChaCha8 stream, so their parity is statistical: the
oracle (test infrastructure, the C++ f64 restatement, camera.rs:302-343) renders
a small frame at a very high spp and stores, per pixel and channel,

  * the mean  (the reference's estimator sum/spp, camera.rs:325-331), and
  * the unbiased per-sample variance of the spp path samples,

as little-endian f32 W x H x 3 (Rgb32FImage layout).  tests/test_stat_parity.py
compares GPU renders against these: per-channel image mean within 0.5 % and
chi^2/N of per-pixel z in [0.9, 1.1].  Jittered pixels make every pixel the
mean over its own viewport square, so a W x H frame is also the block average
of any (kW) x (kH) frame: the full-size C5 check uses the same fixture.

    python scripts/make_stat_fixtures.py [name ...]      (~2 minutes on 8 cores)
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

# name -> (scene, W, H, spp)
CASES = {
    "cornell_32": ("scenes/cornell-box-scene.json", 32, 32, 262144),
    "teapot_32": ("scenes/utah-teapot-scene.json", 32, 32, 16384),
    "earth_48": ("scenes/earth.toml", 48, 27, 262144),
}
INPUTS = {
    "scenes/cornell-box-scene.json": ["scenes/cornell-box-model.json", "scenes/cube-model.toml"],
    "scenes/utah-teapot-scene.json": ["scenes/utah-teapot-model.toml"],
    "scenes/earth.toml": ["scenes/textures/earth.jpg", "scenes/textures/moon.jpg"],
}
OUT = os.path.join(ROOT, "tests", "golden", "stat")


def sha256(path):
    with open(path, "rb") as fh:
        return hashlib.sha256(fh.read()).hexdigest()


def main(names):
    helpers.ensure_oracle()
    os.makedirs(OUT, exist_ok=True)
    mpath = os.path.join(OUT, "manifest.json")
    manifest = {"note": "oracle (f64, ChaCha8 reference stream) high-spp renders: per-pixel mean and unbiased "
                        "per-sample variance, little-endian f32 W x H x 3; made by scripts/make_stat_fixtures.py",
                "cases": {}}
    if os.path.exists(mpath):
        with open(mpath) as fh:
            manifest["cases"].update(json.load(fh).get("cases", {}))
    for name in names or list(CASES):
        scene, w, h, spp = CASES[name]
        t0 = time.time()
        with tempfile.TemporaryDirectory() as td:
            tree, _ = helpers.oracle_tree(scene, td, width=w, height=h, spp=spp)
            img, info, var = helpers.oracle_render(tree, threads=os.cpu_count(), var=True)
        mean_p = os.path.join(OUT, name + ".mean.f32")
        var_p = os.path.join(OUT, name + ".var.f32")
        img.astype("<f4").tofile(mean_p)
        var.astype("<f4").tofile(var_p)
        files = [scene] + INPUTS.get(scene, [])
        manifest["cases"][name] = {
            "scene": scene, "width": w, "height": h, "spp": spp, "rng": "chacha8", "precision": "f64",
            "inputs": {f: sha256(os.path.join(helpers.GOLDEN, f)) for f in files},
            "mean": name + ".mean.f32", "mean_sha256": sha256(mean_p),
            "var": name + ".var.f32", "var_sha256": sha256(var_p),
            "channel_mean": [float(img[c::3].astype("f8").mean()) for c in range(3)],
            "oracle_seconds": round(time.time() - t0, 1), "oracle_threads": info.get("threads")}
        print(name, w, h, spp, manifest["cases"][name]["channel_mean"], f"{time.time() - t0:.1f}s", flush=True)
    with open(mpath, "w") as fh:
        json.dump(manifest, fh, indent=1)
        fh.write("\n")


if __name__ == "__main__":
    main(sys.argv[1:])
