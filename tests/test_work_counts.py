"""tests/golden/work_counts.json (SURVEY §8(d) algorithmic work per sample) is what the
counting oracle produces: C1 is sampled in full (every pixel, full spp), so its counts
are deterministic and re-derived exactly here; every config's FLOP figure is the sum
of its event rates times the committed costs."""
import json
import os
import sys

import pytest

from helpers import GOLDEN, ROOT

sys.path.insert(0, os.path.join(ROOT, "scripts"))


def _load():
    with open(os.path.join(GOLDEN, "work_counts.json")) as fh:
        return json.load(fh)


def test_flops_are_rates_times_costs():
    wc = _load()
    for name, c in wc["configs"].items():
        flops = sum(c["per_sample"][k] * cost for k, cost in wc["costs"].items())
        assert flops == pytest.approx(c["flops_per_sample"], rel=1e-5), name
        assert c["rays_per_sample"] >= 1.0, name  # every sample traces its camera ray


def test_c1_counts_rederived():
    import work_counts

    wc = _load()
    scene, w, h, _, spp, stride = work_counts.CONFIGS["C1"]
    assert stride == 1 and spp == wc["configs"]["C1"]["full_spp"]
    r = work_counts.count(scene, w, h, spp, stride)
    assert r["samples"] == wc["configs"]["C1"]["samples"]
    assert r["per_sample"] == wc["configs"]["C1"]["per_sample"]


def test_bench_work_block():
    sys.path.insert(0, ROOT)
    import bench

    c5 = bench.load_work(bench.DEFAULT_SCENE, 1024, 1024)
    assert c5["name"] == "C5"
    blk = bench.work_block(c5, 1000.0, "f32")
    assert blk["rays_per_s"] == pytest.approx(c5["rays_per_sample"] * 1e9, rel=1e-6)
    assert 0 < blk["valu_flop_frac"] < 1
    # another size of a counted scene takes that scene's per-sample counts and says so
    other = bench.load_work(bench.DEFAULT_SCENE, 100, 100)
    assert other["counted_at"] in ("512x512", "1024x1024") and other["scene"] == bench.DEFAULT_SCENE
    assert bench.load_work("scenes/quads.toml", 100, 100) is None
    # SURVEY §8(d) texel bytes at the bytes per texel as stored, by the formats the scene's images use
    # (nrt_scene_stats.texel_formats: bit 1 << f, f = RGB32F 0, RGBA8 1, RGB8T 2, PAL16 3)
    assert bench.texel_payload_bytes({"texels": 40, "texel_bytes": 128, "texel_formats": 1 << 2}) == 3
    assert bench.texel_payload_bytes({"texels": 4194304, "texel_bytes": 9437184, "texel_formats": 1 << 3}) == 2
    assert bench.texel_payload_bytes({"texels": 32, "texel_bytes": 128, "texel_formats": 1 << 1}) == 4
    assert bench.texel_payload_bytes({"texels": 4, "texel_bytes": 48, "texel_formats": 1 << 0}) == 12
    assert bench.texel_payload_bytes({"texels": 8, "texel_bytes": 60, "texel_formats": (1 << 3) | (1 << 2)}) == 3
    assert bench.texel_payload_bytes({"texels": 0, "texel_bytes": 0, "texel_formats": 0}) == 0
    c3 = bench.load_work("scenes/earth.toml", 1920, 1080)
    assert c3["name"] == "C3" and c3["per_sample"]["texel_fetches"] > 0.2


def test_bench_chooses_the_n_gpu_path():
    """bench.py --gpus N as a driver may invoke it: without a launcher and with RCCL the library's
    multi-GPU render (one process); with --backend gloo, or under torch.distributed.run, one process
    per GPU (started as a child when there is no launcher); N = 1 the single-device path."""
    sys.path.insert(0, ROOT)
    import bench

    c = lambda argv, launched=False: bench.choose_path(bench.parse_args(argv), launched)  # noqa: E731
    assert c([]) == "ranks"
    assert c(["--gpus", "8"]) == "library"
    assert c(["--gpus", "8"], launched=True) == "ranks"
    assert c(["--gpus", "2", "--backend", "gloo"]) == "launch"
    assert c(["--gpus", "2", "--multi", "ranks"]) == "launch"
    assert c(["--gpus", "1", "--multi", "library"]) == "library"
    with pytest.raises(SystemExit):
        c(["--gpus", "2", "--multi", "library"], launched=True)
