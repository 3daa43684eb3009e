#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: Msamples/s on cornell-box-scene.json at
1024x1024, spp=256, over 1/2/4/8 GPUs.

One "step" = one full render of the frame: every rank renders the image rows
y = rank (mod N) with the HIP megakernel (libnrt.so, inputs already resident in
HBM), then one RCCL gather (torch.distributed "nccl" backend = RCCL over xGMI)
brings the rows to rank 0, which un-permutes them into the final framebuffer in
HBM.  The frame is fixed as N grows, so scaling is "strong".

    python bench.py [--gpus N --steps K --warmup W]
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints one JSON line.  The roofline block reports the render kernel's
achieved HBM bandwidth (algorithmic bytes / kernel time, HIP events on the
launch stream) against the 8 TB/s gfx950 peak; PMC-counted traffic comes from
the committed rocprofv3 summary when present.  The cpu_baseline leg times the
oracle (the C++ f64 restatement; the Rust reference cannot be built here) on a
bounded row sample of the same frame.
"""
import argparse
import json
import os
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "nr-ray-tracer_amd"))

METRIC = "Msamples/sec on Cornell box 1024x1024 spp=256; 1/2/4/8-GPU scaling"
DEFAULT_SCENE = "scenes/cornell-box-scene.json"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
VALU_PEAK_TFLOPS = {"f32": 157.3, "f64": 78.6}

# device record sizes (device_scene.hpp) for the algorithmic byte count
REC = {"f32": dict(node=32, prim=80, xform=112), "f64": dict(node=64, prim=144, xform=208)}


def scene_bytes(stats, precision):
    r = REC[precision]
    return (stats["nodes"] * r["node"] + stats["prims"] * r["prim"] + stats["xforms"] * r["xform"]
            + stats["instances"] * 16 + stats["materials"] * 16 + stats["textures"] * 64 + stats["texels"] * 12)


def cpu_baseline(args, samples_note):
    """Oracle (test infrastructure) timed on the host cores over a row sample."""
    sys.path.insert(0, ROOT)
    from oracle import scene_tree

    oracle_bin = os.path.join(ROOT, "oracle", "build", "oracle")
    if not os.path.exists(oracle_bin):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
    threads = min(16, os.cpu_count() or 1)
    with tempfile.TemporaryDirectory() as td:
        old = os.getcwd()
        os.chdir(os.path.join(ROOT, "tests", "golden"))
        try:
            cli = scene_tree.CameraConfig(width=args.width, height=args.height, samples_per_pixel=args.spp)
            text, _ = scene_tree.build_tree(args.scene, cli, td)
        finally:
            os.chdir(old)
        tree = os.path.join(td, "scene.tree")
        with open(tree, "w") as fh:
            fh.write(text)
        stride = args.cpu_row_stride
        out = os.path.join(td, "img.f32")
        st = os.path.join(td, "stats.json")
        subprocess.run([oracle_bin, "render", tree, out, "--threads", str(threads), "--rows", "0", str(stride),
                        "--stats", st], check=True, capture_output=True)
        with open(st) as fh:
            info = json.load(fh)
    rows = (args.height + stride - 1) // stride
    return {"value": round(info["msamples_per_s"], 4), "unit": "Msamples/s", "cores": info["threads"],
            "kind": "port",
            "sample": f"rows y%{stride}==0 of {args.width}x{args.height} at spp={args.spp} ({rows} rows, "
                      f"{info['samples'] / 1e6:.1f} Msamples, {info['seconds']:.1f} s); oracle = C++ f64 "
                      f"restatement, per-pixel dynamic scheduling; Rust reference unbuildable (no toolchain)"}


def load_pmc(precision, rng):
    """The committed rocprofv3 PMC summary of this kernel variant (profiles/pmc_summary.json), or {}."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return {}
    try:
        with open(path) as fh:
            return json.load(fh).get(f"{precision}_{rng}", {}) or {}
    except Exception:
        return {}


def load_work(scene, w, h):
    """Per-sample algorithmic work of this config (tests/golden/work_counts.json), or None."""
    path = os.path.join(ROOT, "tests", "golden", "work_counts.json")
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        wc = json.load(fh)
    for name, c in wc["configs"].items():
        if c["scene"] == scene and c["width"] == w and c["height"] == h:
            return dict(c, name=name)
    return None


def work_block(wc, msamples_per_s, precision):
    """rays/s and the algorithmic VALU-FLOP fraction (oracle event counts x SURVEY §8(d) costs)."""
    if wc is None:
        return None
    tflops = wc["flops_per_sample"] * msamples_per_s * 1e6 / 1e12
    return {"rays_per_s": round(wc["rays_per_sample"] * msamples_per_s * 1e6, 1),
            "rays_per_sample": wc["rays_per_sample"], "flops_per_sample": wc["flops_per_sample"],
            "algorithmic_tflops": round(tflops, 3), "valu_peak_tflops": VALU_PEAK_TFLOPS[precision],
            "valu_flop_frac": round(tflops / VALU_PEAK_TFLOPS[precision], 4),
            "source": f"tests/golden/work_counts.json[{wc['name']}] (oracle event counts, ChaCha8 stream)"}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--scene", default=DEFAULT_SCENE)
    ap.add_argument("--width", type=int, default=1024)
    ap.add_argument("--height", type=int, default=1024)
    ap.add_argument("--spp", type=int, default=256)
    ap.add_argument("--precision", default="f32", choices=["f32", "f64"])
    ap.add_argument("--rng", default="philox", choices=["chacha8", "philox"])
    ap.add_argument("--trace", default="auto", choices=["auto", "bvh", "world-list", "world-bvh"],
                    help="f32 kernel traversal (nrt_trace): auto = world-space list for small flattenable scenes")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-row-stride", type=int, default=16)
    args = ap.parse_args()

    import torch
    import torch.distributed as dist
    import nrt

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and not (world == 1 and args.gpus == 1):
        if world == 1:
            raise SystemExit(f"--gpus {args.gpus} needs torch.distributed.run with {args.gpus} processes")
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    if world > 1:
        dist.init_process_group("nccl", device_id=dev)

    old = os.getcwd()
    os.chdir(os.path.join(ROOT, "tests", "golden"))  # scene files use CWD-relative paths
    try:
        t0 = time.perf_counter()
        scene = nrt.Scene.load(args.scene, nrt.CameraConfig(width=args.width, height=args.height,
                                                              samples_per_pixel=args.spp))
        t_load = time.perf_counter() - t0
    finally:
        os.chdir(old)
    cam = scene.camera
    W, H, spp = cam.width, cam.height, cam.samples_per_pixel
    t0 = time.perf_counter()
    scene.upload(local)
    t_upload = time.perf_counter() - t0

    from nrt import shard

    rows_max = shard.rows_max(H, world)
    rows = scene.rows_selected(H, rank, world)
    assert rows == shard.rows_of(H, rank, world)
    buf = torch.zeros((rows_max, W, 3), dtype=torch.float32, device=dev)
    final = torch.empty((H, W, 3), dtype=torch.float32, device=dev) if (rank == 0 and world > 1) else None
    stream = torch.cuda.current_stream()
    ev = []

    def step(timed):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(stream)
        scene.render_device(buf.data_ptr(), rows * W * 3, precision=args.precision, rng=args.rng, device=local,
                            row_offset=rank, row_stride=world, stream=stream.cuda_stream, trace=args.trace)
        e1.record(stream)
        if timed:
            ev.append((e0, e1))
        if world > 1:  # the single RCCL collective + un-permute on rank 0
            shard.gather_frame(buf, H, dist, rank, world, out=final)

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in ev) / max(len(ev), 1)
    if world > 1:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])

    if rank == 0:
        samples = float(W) * H * spp
        value = samples * args.steps / elapsed / 1e6
        st = scene.stats()
        alg_bytes = rows * W * 12 + scene_bytes(st, args.precision)
        achieved = alg_bytes / (kern_ms / 1e3) / 1e9
        pmc = load_pmc(args.precision, args.rng) if args.scene == DEFAULT_SCENE else {}
        traffic = pmc.get("hbm_bytes_per_launch")
        out = {
            "metric": METRIC, "value": round(value, 3), "unit": "Msamples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
            "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": args.precision,
            "data": "reference scene file scenes/cornell-box-scene.json (no dataset; scene is the input)",
            "config": {"workload": f"{os.path.basename(args.scene)} {W}x{H} spp={spp}", "scene": args.scene,
                       "width": W, "height": H, "spp": spp, "ray_max_bounces": cam.ray_max_bounces,
                       "rng": args.rng, "precision": args.precision, "trace": args.trace,
                       "world_prims": st["world_prims"],
                       "parallelism": f"rows interleaved over {world} GPU(s), one RCCL gather to rank 0"},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 6), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": traffic,
                         "kernel_ms": round(kern_ms, 3), "algorithmic_bytes_per_launch": alg_bytes,
                         "note": "path is VALU-issue-bound (no dense contraction, no MFMA); HBM fraction is "
                                 "reported as the north star asks",
                         "valu_issue_frac": pmc.get("valu_issue_frac"),
                         "valu_lane_utilization": pmc.get("valu_lane_utilization"),
                         "pmc_source": "profiles/pmc_summary.json" if pmc else None},
            "work": work_block(load_work(args.scene, W, H), value, args.precision),
            "timings_s": {"scene_load_and_bvh": round(t_load, 4), "upload": round(t_upload, 4)},
        }
        if not args.no_cpu_baseline and world == 1:
            out["cpu_baseline"] = cpu_baseline(args, None)
        elif not args.no_cpu_baseline:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
