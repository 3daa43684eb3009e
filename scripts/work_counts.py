"""Algorithmic work per sample for the SURVEY §8(d) configs -> tests/golden/work_counts.json.

The oracle (test infrastructure, C++ f64 restatement) built with event counters
(oracle/build/oracle_stats) renders a bounded sample of each config with the
reference's ChaCha8 stream; the counts divided by the samples rendered are the
per-sample event rates.  FLOPs per sample = sum(rate x cost) with the per-event
costs of SURVEY §8(d) (aabb.rs:116-129, sphere.rs:110-161, plane.rs:142-168,
rotate/scale/translate, camera.rs:236-300).  bench.py reads the committed JSON
(data only) to report rays/s and the VALU-FLOP fraction beside the HBM roofline.

    python scripts/work_counts.py            # all configs (~2 min on 8 cores)
"""
import json
import os
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))

import helpers  # noqa: E402

# SURVEY §8(d) per-event FLOP costs
COSTS = {"aabb_tests": 24, "sphere_tests": 31, "sphere_hits": 27, "plane_tests": 51, "transform_enters": 30,
         "scatters": 30, "camera_rays": 25}

# config -> (scene, W, H, full spp, sampled spp, row stride of the sample)
CONFIGS = {
    "C1": ("scenes/spheres.toml", 400, 225, 16, 16, 1),
    "C2": ("scenes/cornell-box-scene.json", 512, 512, 64, 64, 1),
    "C3": ("scenes/earth.toml", 1920, 1080, 128, 8, 1),
    "C4": ("scenes/utah-teapot-scene.json", 1024, 1024, 256, 8, 1),
    "C5": ("scenes/cornell-box-scene.json", 1024, 1024, 256, 32, 1),
}


def count(scene, w, h, spp, stride):
    with tempfile.TemporaryDirectory() as td:
        tree, _ = helpers.oracle_tree(scene, td, width=w, height=h, spp=spp)
        _, info = helpers.oracle_render(tree, threads=os.cpu_count(), rows=(0, stride), stats=True)
    n = info["samples"]
    rates = {k: info[k] / n for k in ("aabb_tests", "sphere_tests", "sphere_hits", "plane_tests", "plane_hits",
                                        "transform_enters", "rays", "scatters", "camera_rays", "texel_fetches")}
    flops = sum(rates[k] * c for k, c in COSTS.items())
    return {"scene": scene, "width": w, "height": h, "sampled_spp": spp, "row_stride": stride, "samples": n,
            "per_sample": {k: round(v, 6) for k, v in rates.items()}, "rays_per_sample": round(rates["rays"], 6),
            "flops_per_sample": round(flops, 3), "texel_bytes_per_sample": round(12 * rates["texel_fetches"], 4)}


def main():
    helpers.ensure_oracle()
    out = {"note": "oracle_stats (ChaCha8 stream, f64) over a bounded sample of each config; rays = traced segments "
                   "(get_ray_color calls past the depth cap, camera.rs:269-300); flops = sum(rate x cost)",
           "costs": COSTS, "configs": {}}
    for name, (scene, w, h, full, spp, stride) in CONFIGS.items():
        r = count(scene, w, h, spp, stride)
        r["full_spp"] = full
        out["configs"][name] = r
        print(name, r["rays_per_sample"], "rays/sample", r["flops_per_sample"], "flops/sample", flush=True)
    path = os.path.join(ROOT, "tests", "golden", "work_counts.json")
    with open(path, "w") as fh:
        json.dump(out, fh, indent=1)
        fh.write("\n")


if __name__ == "__main__":
    main()
