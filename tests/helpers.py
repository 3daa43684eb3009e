"""Shared test helpers: the oracle (test infrastructure) and scene fixtures."""
import contextlib
import os
import subprocess
import tempfile

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
GOLDEN = os.path.join(ROOT, "tests", "golden")
SCENES = os.path.join(GOLDEN, "scenes")
ORACLE_BIN = os.path.join(ROOT, "oracle", "build", "oracle")
ORACLE_STATS_BIN = os.path.join(ROOT, "oracle", "build", "oracle_stats")


@contextlib.contextmanager
def in_golden():
    """Scene files reference `scenes/...` relative to the CWD, as in the reference."""
    old = os.getcwd()
    os.chdir(GOLDEN)
    try:
        yield
    finally:
        os.chdir(old)


def ensure_oracle():
    if not os.path.exists(ORACLE_BIN) or not os.path.exists(ORACLE_STATS_BIN):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    return ORACLE_BIN


def is_legacy(scene):
    """Scene files in the legacy index schema (loaded with the explicit opt-in)."""
    return scene.endswith("triangles.toml")


def oracle_tree(scene, workdir, width=None, height=None, spp=None, bounces=None):
    """Independent Python loader -> oracle tree file (path)."""
    from oracle import scene_tree

    cli = scene_tree.CameraConfig(width=width, height=height, samples_per_pixel=spp, ray_max_bounces=bounces)
    with in_golden():
        text, cam = scene_tree.build_tree(scene, cli, workdir, legacy=is_legacy(scene))
    path = os.path.join(workdir, os.path.basename(scene) + ".tree")
    with open(path, "w") as fh:
        fh.write(text)
    return path, cam


def oracle_render(tree, threads=None, rows=(0, 1), stats=False, spp=None, var=False):
    """Run the oracle; returns (image, info) or (image, info, per-sample variance) with var=True."""
    ensure_oracle()
    with tempfile.TemporaryDirectory() as td:
        out = os.path.join(td, "img.f32")
        st = os.path.join(td, "stats.json")
        vp = os.path.join(td, "var.f32")
        cmd = [ORACLE_STATS_BIN if stats else ORACLE_BIN, "render", tree, out, "--rows", str(rows[0]), str(rows[1]),
               "--stats", st]
        if var:
            cmd += ["--var", vp]
        if threads:
            cmd += ["--threads", str(threads)]
        if spp:
            cmd += ["--spp", str(spp)]
        subprocess.run(cmd, check=True, capture_output=True)
        import json
        img = np.fromfile(out, dtype="<f4")
        with open(st) as fh:
            info = json.load(fh)
        if var:
            return img, info, np.fromfile(vp, dtype="<f4")
        return img, info


def oracle_dump(tree):
    ensure_oracle()
    return subprocess.run([ORACLE_BIN, "dump", tree], check=True, capture_output=True, text=True).stdout
