#!/usr/bin/env python3
"""bench.py — BASELINE.json metric: Msamples/s on cornell-box-scene.json at
1024x1024, spp=256, over 1/2/4/8 GPUs.

One "step" = one full frame, ending with the framebuffer in host memory (the
reference times `scene.render`, which returns a host `Rgb32FImage`,
app/commands/render.rs:57-62, camera.rs:342):

  * every GPU renders the image rows y = r (mod N) with the HIP megakernel
    (libnrt.so; the scene is resident in HBM since upload),
  * N > 1: one RCCL gather (over xGMI) of the row buffers to the first GPU, which
    un-permutes them into the frame in HBM,
  * the first GPU's frame is copied to pinned host memory on a copy stream.  Frames
    are double-buffered, so frame k's device-to-host copy overlaps frame k+1's render
    (as a render loop would run); the timed region ends when the last frame is
    on the host.

Two ways to run N > 1, both the same frame bit for bit (frame_sha256 on the line):
  * one process (`python bench.py --gpus N`, no launcher): the library's own multi-GPU
    render, nrt_render_opts.gpus = N (csrc/multi.hip: ncclCommInitAll over the N devices,
    one ncclGather per frame) -- what a host calling the C ABI gets;
  * one process per GPU (`python -m torch.distributed.run --nproc-per-node N ... bench.py
    --gpus N`): rank r renders its rows, torch.distributed's "nccl" (= RCCL) gathers them
    to rank 0 (nrt/shard.py).  `--backend gloo` without a launcher starts that launcher as
    a child process (never exec) and forwards its line and exit status.

The frame is fixed as N grows, so scaling is "strong".

    python bench.py [--gpus N --steps K --warmup W]      # N > 1: the library's multi-GPU render
    python -m torch.distributed.run --nproc-per-node N ... bench.py --gpus N ...

Rank 0 prints one JSON line.  `roofline` prices the render kernel against the
bound that limits it, the FP32 (or FP64) VALU peak: achieved = SURVEY §8(d)'s
algorithmic FLOPs per sample (oracle event counts x per-event costs,
tests/golden/work_counts.json) x samples per launch / the kernel's HIP-event
time on its launch stream.  The HBM figures the north star asks for sit beside
it (`roofline.hbm`): framebuffer + texel fetch bytes per launch over the same time,
and rocprofv3 FETCH_SIZE/WRITE_SIZE traffic from profiles/pmc_summary.json,
looked up by (scene, size, spp, precision, rng, trace).  The cpu_baseline leg
times the oracle (the C++ f64 restatement; the Rust reference cannot be built
here), compiled for the host CPU, on every core this process may use, over a
bounded row sample of the same frame.
"""
import argparse
import hashlib
import json
import math
import os
import platform
import subprocess
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "nr-ray-tracer_amd"))

METRIC = "Msamples/sec on Cornell box 1024x1024 spp=256; 1/2/4/8-GPU scaling"
DEFAULT_SCENE = "scenes/cornell-box-scene.json"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)
VALU_PEAK_TFLOPS = {"f32": 157.3, "f64": 78.6}  # 256 CUs x 2.4 GHz (vendor figures)

# device record sizes (device_scene.hpp) for the algorithmic byte count
REC = {"f32": dict(node=32, prim=80, xform=112), "f64": dict(node=64, prim=144, xform=208)}


def scene_bytes(stats, precision):
    r = REC[precision]
    return (stats["nodes"] * r["node"] + stats["prims"] * r["prim"] + stats["xforms"] * r["xform"]
            + stats["instances"] * 16 + stats["materials"] * 16 + stats["textures"] * 64 + stats["texel_bytes"])


# ------------------------------------------------------------------ CPU baseline

def host_cpus():
    """(cores this process may run on, description): the affinity set, capped by a cgroup CPU quota."""
    aff = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max",):
        try:
            with open(path) as fh:
                q, p = fh.read().split()[:2]
            if q != "max":
                quota = float(q) / float(p)
        except (OSError, ValueError):
            pass
    cores = aff if quota is None else max(1, min(aff, int(math.floor(quota + 1e-9))))
    model = platform.processor() or ""
    try:
        with open("/proc/cpuinfo") as fh:
            for line in fh:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    desc = f"{model}; os.cpu_count()={os.cpu_count()}, affinity={aff}, cgroup quota={quota if quota else 'none'}"
    return cores, model, desc


def native_oracle():
    """The oracle compiled for this host's CPU (-march=native; same IEEE arithmetic, -ffp-contract=off),
    cached per CPU model; the portable in-tree build if no compiler is available."""
    _, model, _ = host_cpus()
    tag = hashlib.sha256(model.encode()).hexdigest()[:12]
    path = os.path.join(ROOT, "oracle", "build", f"oracle_native_{tag}")
    if not os.path.exists(path):
        os.makedirs(os.path.dirname(path), exist_ok=True)
        r = subprocess.run(["g++", "-std=c++17", "-O3", "-march=native", "-ffp-contract=off", "-fno-fast-math",
                            "-pthread", "-o", path, os.path.join(ROOT, "oracle", "oracle.cpp")],
                           capture_output=True)
        if r.returncode != 0:
            path = os.path.join(ROOT, "oracle", "build", "oracle")
            if not os.path.exists(path):
                subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "oracle")], check=True)
            return path, "portable -O3 build (g++ -march=native failed)"
    return path, "g++ -O3 -march=native -ffp-contract=off"


def cpu_baseline(args):
    """Oracle (test infrastructure) timed on the host cores over a row sample."""
    sys.path.insert(0, ROOT)
    from oracle import scene_tree

    oracle_bin, build = native_oracle()
    threads, _, desc = host_cpus()
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
                      f"{info['samples'] / 1e6:.1f} Msamples, {info['seconds']:.2f} s wall, "
                      f"{info['seconds'] * info['threads']:.1f} CPU-s); oracle = C++ f64 restatement of the "
                      f"reference path ({build}), per-pixel dynamic scheduling over all usable cores; "
                      f"Rust reference unbuildable (no toolchain)",
            "cpu": desc}


# ------------------------------------------------------------------ committed evidence lookups

def load_pmc(key):
    """The committed rocprofv3 summary of exactly this kernel variant and config, or {}."""
    path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    if not os.path.exists(path):
        return {}
    try:
        with open(path) as fh:
            entries = json.load(fh).get("entries", [])
    except Exception:
        return {}
    for e in entries:
        if all(e.get(k) == v for k, v in key.items()):
            return e
    return {}


def load_work(scene, w, h, spp=None):
    """Per-sample algorithmic work of this config (tests/golden/work_counts.json), or None.
    Per-sample counts do not depend on spp (samples of a pixel are independent).  Another image size of
    a counted scene (same camera, the view sampled more or less densely) takes that scene's counts and
    says so in `counted_at`."""
    path = os.path.join(ROOT, "tests", "golden", "work_counts.json")
    if not os.path.exists(path):
        return None
    with open(path) as fh:
        wc = json.load(fh)
    same_scene = None
    for name, c in wc["configs"].items():
        if c["scene"] == scene and c["width"] == w and c["height"] == h:
            return dict(c, name=name)
        if c["scene"] == scene and same_scene is None:
            same_scene = dict(c, name=name, counted_at=f"{c['width']}x{c['height']}")
    return same_scene


# bytes a texel fetch reads as stored, per format (nrt_scene_stats.texel_formats bit 1 << f; device_scene.hpp
# TEXFMT_*): RGB32F 12, RGBA8 4, RGB8T 3, PAL16 2 (the index; its palette word stays in the L2)
TEXEL_FETCH_BYTES = {0: 12, 1: 4, 2: 3, 3: 2}


def texel_payload_bytes(stats):
    """Bytes per texel fetch as stored (2 / 3 / 4 / 12) of the scene's image textures (the largest, if
    they use several formats); 0 without image textures."""
    mask = stats.get("texel_formats", 0)
    if not stats.get("texels") or not mask:
        return 0
    return max(b for f, b in TEXEL_FETCH_BYTES.items() if mask & (1 << f))


def work_block(wc, msamples_per_s, precision):
    """rays/s and the algorithmic VALU-FLOP rate of a whole-job throughput (oracle event counts x
    SURVEY §8(d) per-event costs)."""
    if wc is None:
        return None
    tflops = wc["flops_per_sample"] * msamples_per_s * 1e6 / 1e12
    return {"rays_per_s": round(wc["rays_per_sample"] * msamples_per_s * 1e6, 1),
            "rays_per_sample": wc["rays_per_sample"], "flops_per_sample": wc["flops_per_sample"],
            "algorithmic_tflops": round(tflops, 3), "valu_peak_tflops": VALU_PEAK_TFLOPS[precision],
            "valu_flop_frac": round(tflops / VALU_PEAK_TFLOPS[precision], 4),
            "source": f"tests/golden/work_counts.json[{wc['name']}] (oracle event counts, ChaCha8 stream"
                      + (f"; counted at {wc['counted_at']}, the same view)" if wc.get("counted_at") else ")")}


# ------------------------------------------------------------------ main

def parse_args(argv=None):
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
    ap.add_argument("--backend", default="nccl", choices=["nccl", "gloo"],
                    help="one process per GPU: nccl = RCCL over xGMI, one GPU per rank (the measured path); gloo = "
                         "host-side gather, ranks may share a GPU (rehearses the N > 1 step on a one-GPU box)")
    ap.add_argument("--multi", default="auto", choices=["auto", "library", "ranks"],
                    help="library = one process, the library's multi-GPU render (nrt_render_opts.gpus, RCCL inside "
                         "libnrt.so; at N = 1 too, through the same RCCL code); ranks = one process per GPU under "
                         "torch.distributed.run (started as a child process when this one has no launcher); auto = "
                         "ranks under a launcher or with --backend gloo, library for N > 1 without a launcher, else "
                         "the single-device path")
    ap.add_argument("--cpu-only", action="store_true",
                    help="time only the CPU baseline (the oracle on the host cores) for this config, e.g. BASELINE C1; "
                         "prints one JSON line, no GPU is touched")
    ap.add_argument("--pipeline", type=int, default=None,
                    help="frames whose renders may be in flight at once: consecutive renders rotate over this many "
                         "HIP streams and row buffers, so frame k+1's workgroups take the SIMDs frame k's last paths "
                         "leave idle (each frame is still one full render; ms_per_step = elapsed / steps); 1 (or 0): "
                         "each render waits for the previous one.  Default 3 on one GPU, 2 with N > 1 (the gathers' "
                         "streams share the process's 4 hardware queues)")
    ap.add_argument("--kernel-only", action="store_true",
                    help="diagnostics (PMC passes): no device-to-host copy of the frame, so device-wide counters "
                         "sampled over a render dispatch see the render kernel alone")
    return ap.parse_args(argv)


def launch_ranks_child(args):
    """`--gpus N` one process per GPU without a launcher: torch.distributed.run as a CHILD process (this
    process has not touched the GPU), its output passed through, its exit status returned."""
    import socket

    with socket.socket() as sk:  # a free rendezvous port on the loopback
        sk.bind(("127.0.0.1", 0))
        port = sk.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    env.setdefault("OMP_NUM_THREADS", "1")
    return subprocess.run(cmd, env=env).returncode


def load_scene(args, nrt):
    old = os.getcwd()
    os.chdir(os.path.join(ROOT, "tests", "golden"))  # scene files use CWD-relative paths
    try:
        t0 = time.perf_counter()
        scene = nrt.Scene.load(args.scene, nrt.CameraConfig(width=args.width, height=args.height,
                                                              samples_per_pixel=args.spp))
        return scene, time.perf_counter() - t0
    finally:
        os.chdir(old)


def kernel_variant_of(jit_before, jit_after, steps, mixed=False):
    specialised = jit_after["launches"] - jit_before["launches"] >= steps
    variant = "scene-specialised (hiprtc)" if specialised else "generic"
    if mixed:
        variant = "MIXED over ranks (scene-specialised on some, generic on others)"
        print("bench.py: WARNING: ranks ran different kernel variants", file=sys.stderr, flush=True)
    if jit_after["failed"]:
        variant = "generic (scene-specialised build FAILED)"
        print(f"bench.py: WARNING: {jit_after['failed']} scene-specialised kernel build(s) failed; the generic "
              f"kernel was timed", file=sys.stderr, flush=True)
    return variant


def report(args, nrt, scene, *, n_gpus, rows, elapsed, kern_ms, d2h_ms, timings_s, frame_sha, jit_before, jit_after,
           kernel_variant, parallelism, extra=None):
    """The JSON line.  `rows` / `kern_ms`: the rows and HIP-event time of the launch the roofline prices
    (the first GPU's)."""
    cam = scene.camera
    W, H, spp = cam.width, cam.height, cam.samples_per_pixel
    samples = float(W) * H * spp
    value = samples * args.steps / elapsed / 1e6
    st = scene.stats()
    key = {"scene": args.scene, "width": W, "height": H, "spp": spp, "precision": args.precision,
           "rng": args.rng, "trace": args.trace, "n_gpus": n_gpus}
    pmc = load_pmc(key)
    traffic = pmc.get("hbm_bytes_per_launch")
    wc = load_work(args.scene, W, H, spp)
    # SURVEY §8(d) bytes per sample: 12/spp of framebuffer + texel_fetches/sample x the texel's bytes as
    # stored (PAL16: the 2-byte index); the scene's records are a cache-resident working set, listed
    # beside it (scene_bytes)
    fb_bytes = rows * W * 12
    texel_b = texel_payload_bytes(st)
    fetches = 0.0 if wc is None else wc["per_sample"].get("texel_fetches", 0.0)
    tex_bytes = fetches * texel_b * rows * W * spp
    alg_bytes = fb_bytes + tex_bytes
    hbm_achieved = alg_bytes / (kern_ms / 1e3) / 1e9
    # the profiled kernel's time per launch: the steady period of the trace (scripts/trace_period.py; with frames
    # in flight a dispatch's begin..end also spans its wait behind the ones ahead), else the stats' average
    prof_s = (pmc.get("steady_period_ns") or pmc.get("avg_ns", 0)) / 1e9 if pmc else 0
    counter_gbs = traffic / prof_s / 1e9 if traffic and prof_s else None
    peak = VALU_PEAK_TFLOPS[args.precision]
    if wc is not None:
        flops_launch = wc["flops_per_sample"] * rows * W * spp  # this GPU's launch
        achieved = flops_launch / (kern_ms / 1e3) / 1e12
    else:
        flops_launch, achieved = None, None
    out = {
        "metric": METRIC, "value": round(value, 3), "unit": "Msamples/s", "n_gpus": n_gpus,
        "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(elapsed / args.steps * 1e3, 3),
        "higher_is_better": True, "scaling": "strong", "vs_baseline": None, "dtype": args.precision,
        "data": "reference scene file scenes/cornell-box-scene.json (no dataset; scene is the input)",
        "config": {"workload": f"{os.path.basename(args.scene)} {W}x{H} spp={spp}", "scene": args.scene,
                   "width": W, "height": H, "spp": spp, "ray_max_bounces": cam.ray_max_bounces,
                   "rng": args.rng, "precision": args.precision, "trace": args.trace,
                   "world_prims": st["world_prims"], "parallelism": parallelism,
                   "timed_step": "render + (N>1) gather/un-permute" + (
                       " (--kernel-only diagnostics: no device-to-host copy)" if args.kernel_only else
                       " + device-to-host copy of the frame (pinned, double-buffered: frame k's copy overlaps "
                       "frame k+1's render)")},
        "roofline": {
            "bound": "valu", "achieved": None if achieved is None else round(achieved, 3), "peak": peak,
            "unit": "TFLOP/s", "frac": None if achieved is None else round(achieved / peak, 4),
            "traffic": traffic,
            "flops_per_launch": flops_launch, "kernel_ms": round(kern_ms, 3),
            "kernel_ms_basis": "device time per frame: the first timed render's start to the last render's end, over "
                               "the frames (HIP events); frames in flight overlap, so a dispatch's own begin..end "
                               "(rocprofv3 --stats AverageNs) also spans its wait behind the frames ahead: compare "
                               "with scripts/trace_period.py's steady period of the same trace "
                               "(profiles/*_trace_period.json, pmc.steady_period_ns)",
            "flops_source": None if wc is None else
            f"tests/golden/work_counts.json[{wc['name']}]: {wc['flops_per_sample']} algorithmic FLOPs/sample "
            f"(oracle event counts x SURVEY §8(d) per-event costs) x {rows * W * spp} samples per launch",
            "hbm": {"achieved": round(hbm_achieved, 6), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                    "frac": hbm_achieved / HBM_PEAK_GBS, "algorithmic_bytes_per_launch": round(alg_bytes),
                    "algorithmic_bytes": {"framebuffer": fb_bytes, "texels": round(tex_bytes),
                                          "texel_fetches_per_sample": fetches, "bytes_per_texel": texel_b,
                                          "source": "SURVEY §8(d): 12/spp + texel_fetches x bytes per "
                                                    "texel as stored, per sample"},
                    "scene_bytes": scene_bytes(st, args.precision),
                    "traffic": traffic,
                    # rocprofv3 FETCH_SIZE + WRITE_SIZE per launch over the profiled kernel time
                    # (profiles/pmc_summary.json, the committed profile of this variant and config)
                    "counter_gbs": None if counter_gbs is None else round(counter_gbs, 3),
                    "counter_frac": None if counter_gbs is None else counter_gbs / HBM_PEAK_GBS,
                    "traffic_over_algorithmic": None if not traffic else round(traffic / alg_bytes, 3)},
            "pmc": {k: pmc.get(k) for k in ("kernel", "avg_ns", "steady_period_ns", "valu_issue_frac", "valu_lane_utilization",
                                            "valu_busy_est", "wait_inst_frac", "wait_any_frac", "hbm_fetch_bytes",
                                            "hbm_write_bytes", "tcc_hit_rate", "source")} if pmc else None,
            "note": "no dense contraction (no MFMA): the render kernel is bound by VALU issue and lane "
                    "divergence; its compulsory HBM traffic is the framebuffer (plus texel fetches in textured "
                    "scenes)"},
        "work": work_block(wc, value, args.precision),
        "timings_ms": {"kernel_device_only": round(kern_ms, 3), "d2h_copy": round(d2h_ms, 3),
                       "frame_wall": round(elapsed / args.steps * 1e3, 3)},
        # the reference times scene.render (render.rs:57-62): a one-shot render also pays the runtime start,
        # the load, the upload and the scene-specialised kernel's build or disk-cache load, done here before
        # the timed frames and reported on their own; first_frame = scene load start -> first frame on the host
        "timings_s": timings_s,
        "frame_sha256": frame_sha,
        "build_id": nrt.build_id(),  # sha256 prefix of the sources libnrt.so was built from
        # scene-specialised kernels (jit.hip): built with hiprtc or read from the disk cache in this process,
        # renders using one; the timed frames ran on one only if every timed launch counted (a failed build
        # falls back to the generic kernel, which is slower: then the line says so)
        "jit": dict(jit_after, timed_launches=jit_after["launches"] - jit_before["launches"]),
        "kernel_variant": kernel_variant,
    }
    if extra:
        out.update(extra)
    if not args.no_cpu_baseline and n_gpus == 1:
        out["cpu_baseline"] = cpu_baseline(args)
    elif not args.no_cpu_baseline:
        out["cpu_baseline"] = None
    print(json.dumps(out), flush=True)


def run_library(args):
    """One process, N GPUs: the library's multi-GPU render (nrt_render_opts.gpus = N, csrc/multi.hip) into a
    device frame on GPU 0, then the pinned, double-buffered host copy as in the single-device path."""
    import torch
    import nrt

    N = args.gpus
    ndev = torch.cuda.device_count()
    if N > ndev:
        raise SystemExit(f"--gpus {N} --multi library: {ndev} GPU(s) visible")
    t0 = time.perf_counter()
    torch.cuda.set_device(0)
    dev = torch.device("cuda:0")
    torch.zeros(1, device=dev)  # HIP runtime start (reported apart from the scene upload)
    nrt.lib()
    t_init = time.perf_counter() - t0
    scene, t_load = load_scene(args, nrt)
    t_first0 = time.perf_counter() - t_load
    cam = scene.camera
    W, H = cam.width, cam.height
    t0 = time.perf_counter()
    for d in range(N):
        scene.upload(d)
    t_upload = time.perf_counter() - t0
    t0 = time.perf_counter()
    # the library runs GPU 0's gathers and the un-permute on this stream, and the frame's host copy follows
    # them here too: GPU 0 then runs this stream + the library's three render streams, the process's 4
    # hardware queues (GPU_MAX_HW_QUEUES; a fifth stream would share a queue with a render)
    stream = torch.cuda.current_stream()
    scene.prepare(precision=args.precision, rng=args.rng, device=0, trace=args.trace, gpus=N)  # RCCL comms, buffers
    NB = max(2, args.pipeline or 2)  # device / pinned host frames (the library keeps its own buffer sets)
    frames = [torch.empty((H, W, 3), dtype=torch.float32, device=dev) for _ in range(NB)]
    host = [torch.empty((H, W, 3), dtype=torch.float32).pin_memory() for _ in range(NB)]
    cev = []
    torch.cuda.synchronize()
    t_prepare = time.perf_counter() - t0

    def step(k, timed):
        slot = k % NB  # (frames[slot] and host[slot] were last used NB frames ago, earlier on this stream)
        scene.render_device(frames[slot].data_ptr(), H * W * 3, precision=args.precision, rng=args.rng, device=0,
                            stream=stream.cuda_stream, trace=args.trace, gpus=N)
        if not args.kernel_only:
            c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            c0.record(stream)
            host[slot].view(-1).copy_(frames[slot].view(-1), non_blocking=True)
            c1.record(stream)
            if timed:
                cev.append((c0, c1))

    first_frame = None
    for k in range(args.warmup):
        step(k, False)
        if k == 0:
            torch.cuda.synchronize()
            first_frame = time.perf_counter() - t_first0
    torch.cuda.synchronize()
    if args.warmup:
        scene.render_timings()  # (opens the frame-period window: the timed frames' completions follow)
    jit_before = nrt.jit_stats()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k, True)
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    tm = scene.render_timings()  # the last timed frame's per-device kernel and gather times
    d2h_ms = sum(a.elapsed_time(b) for a, b in cev) / max(len(cev), 1) if cev else 0.0
    jit_after = nrt.jit_stats()
    last = host[(args.warmup + args.steps - 1) % NB].numpy()
    frame_sha = None if args.kernel_only else hashlib.sha256(last.tobytes()).hexdigest()
    rows = scene.rows_selected(H, 0, N)
    # the device time per timed frame: GPU 0's first timed render start to the last frame's completion, over
    # the frames (the renders overlap at their ends, as with --pipeline > 1)
    kern_ms = tm["period_ms"] if tm["period_ms"] > 0 else tm["kernel_ms"][0]
    report(args, nrt, scene, n_gpus=N, rows=rows, elapsed=elapsed, kern_ms=kern_ms, d2h_ms=d2h_ms,
           timings_s={"runtime_init": round(t_init, 4), "scene_load_and_bvh": round(t_load, 4),
                      "upload": round(t_upload, 4), "multi_gpu_prepare": round(t_prepare, 4),
                      "jit_compile": jit_after["compile_s"],
                      "first_frame": None if first_frame is None else round(first_frame, 4)},
           frame_sha=frame_sha, jit_before=jit_before, jit_after=jit_after,
           kernel_variant=kernel_variant_of(jit_before, jit_after, args.steps * N),
           parallelism=f"rows interleaved over {N} GPU(s) of one process, one RCCL ncclGather to GPU 0 "
                       f"(libnrt.so nrt_render_opts.gpus)",
           extra={"multi_gpu": {"path": "library", "launch_ms_per_gpu": [round(x, 3) for x in tm["kernel_ms"]],
                                "gather_unpermute_ms": round(tm["gather_ms"], 3),
                                "frame_ms_gpu0": round(tm["period_ms"], 3),
                                "note": "HIP-event times of the last timed frame (nrt_render_timings): each "
                                        "device's launch begin..end (overlapping the previous frame's tail), the "
                                        "gather + un-permute on GPU 0, the device time per timed frame on GPU 0 (first render start to last completion, over the frames)"}})


def main():
    args = parse_args()
    if os.environ.get("NRT_MULTI_LOOPBACK", "0") not in ("", "0") and not os.environ.get("NRT_BENCH_DIAG_LOOPBACK"):
        # the library's test-only loopback (every shard of a gpus = N render on GPU 0, the gather as
        # device copies) would time N shards on one GPU as an N-GPU line: never a measurement
        raise SystemExit("bench.py: NRT_MULTI_LOOPBACK is set (test-only multi-GPU loopback); unset it to measure")
    if args.cpu_only:
        cpu = cpu_baseline(args)
        print(json.dumps({"metric": "Msamples/sec (CPU baseline, oracle)", "value": cpu["value"], "unit": "Msamples/s",
                          "higher_is_better": True, "config": {"workload": f"{os.path.basename(args.scene)} "
                                                               f"{args.width}x{args.height} spp={args.spp}",
                                                               "scene": args.scene, "width": args.width,
                                                               "height": args.height, "spp": args.spp},
                          "cpu_baseline": cpu}), flush=True)
        return 0

    path = choose_path(args, "WORLD_SIZE" in os.environ)
    if path == "library":
        return run_library(args)
    if path == "launch":
        # one process per GPU, no launcher: torch.distributed.run as a child (nothing has touched the GPU)
        return launch_ranks_child(args)
    return run_ranks(args)


def choose_path(args, launched):
    """Which N-GPU step this invocation runs: "library" (one process, nrt_render_opts.gpus), "launch"
    (start torch.distributed.run as a child, one process per GPU), or "ranks" (this process is a rank,
    or N = 1 on the single-device path)."""
    multi = args.multi
    if multi == "auto":
        multi = "ranks" if launched or (args.gpus > 1 and args.backend == "gloo") else (
            "library" if args.gpus > 1 else "ranks")
    if multi == "library":
        if launched:
            raise SystemExit("--multi library runs in one process: start it without torch.distributed.run")
        return "library"
    if not launched and args.gpus > 1:
        return "launch"
    return "ranks"


def run_ranks(args):
    """One process per GPU (N = 1: this process alone): rank r renders rows y = r (mod N); N > 1: one
    torch.distributed gather (RCCL with --backend nccl) to rank 0 and a device un-permute there."""
    import torch
    import torch.distributed as dist
    import nrt
    from nrt import shard

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} under a launcher of {world} process(es)")
    t0 = time.perf_counter()
    ndev = torch.cuda.device_count()
    if args.backend == "nccl" and local >= ndev:
        raise SystemExit(f"rank {rank}: LOCAL_RANK {local} but {ndev} GPU(s) visible (nccl needs one GPU per rank)")
    local = local % ndev  # gloo: ranks may share a GPU
    torch.cuda.set_device(local)
    dev = torch.device(f"cuda:{local}")
    torch.zeros(1, device=dev)  # HIP runtime start (reported apart from the scene upload)
    nrt.lib()
    t_init = time.perf_counter() - t0
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group("gloo")

    scene, t_load = load_scene(args, nrt)
    t_first0 = time.perf_counter() - t_load
    cam = scene.camera
    W, H = cam.width, cam.height
    t0 = time.perf_counter()
    scene.upload(local)
    t_upload = time.perf_counter() - t0

    rows_max = shard.rows_max(H, world)
    rows = scene.rows_selected(H, rank, world)
    assert rows == shard.rows_of(H, rank, world)
    stream = torch.cuda.current_stream()
    lead = rank == 0
    # D = --pipeline row buffers rendered on D streams (D = 1: one stream); N = 1: the row buffers are
    # the frames; N > 1: rank 0 gathers into D frames.  Pinned host frames, one per buffer.
    D = max(1, args.pipeline if args.pipeline is not None else (3 if world == 1 else 2))
    # buffers: at least two, so frame k's host copy overlaps frame k+1's render; N > 1: one more than the
    # render streams, so frame k + D's render waits for frame k - 1's gather, not frame k's: the gather's
    # RCCL kernel finds CU slots only where a later render's persistent workgroups leave (its tail), and
    # with D buffers render k + D would wait for exactly that
    NB = max(2, D) if world == 1 else D + 1
    rbuf = [torch.zeros((rows_max, W, 3), dtype=torch.float32, device=dev) for _ in range(NB)]
    # (N = 1: the current stream is one of them, so D = 3 render streams and the copy stream stay within
    # the process's 4 hardware queues; N > 1: it carries the gathers)
    rstreams = ([stream] if world == 1 or D == 1 else []) + [torch.cuda.Stream(device=dev)
                                                             for _ in range(D - (1 if world == 1 or D == 1 else 0))]
    freed = [None] * NB  # event: rbuf[slot] consumed (copied to the host, or gathered)
    if lead:
        frames = rbuf if world == 1 else [torch.empty((H, W, 3), dtype=torch.float32, device=dev)
                                          for _ in range(NB)]
        host = [torch.empty((H, W, 3), dtype=torch.float32).pin_memory() for _ in range(NB)]
        # D >= 4 on one GPU: each frame's host copy follows its render on the render's own stream (no copy
        # stream: D render streams are all the hardware queues the process has)
        copy_on_render = world == 1 and D >= 4
        copy_stream = None if copy_on_render else torch.cuda.Stream(device=dev)
        copied = [None] * NB
    # HIP creates a stream's hardware queue at its first launch (milliseconds): touch every stream before
    # the timed region even when there are fewer warm-up frames than streams
    for st in rstreams + ([copy_stream] if lead and copy_stream is not None else []):
        with torch.cuda.stream(st):
            torch.zeros(1, device=dev)
    torch.cuda.synchronize()
    rend, cev = [], []
    single = {}

    def step(k, timed, isolated=False):
        slot = k % NB
        rs = rstreams[k % D]
        if freed[slot] is not None:
            rs.wait_event(freed[slot])  # rbuf[slot] was consumed NB frames ago
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(rs)
        scene.render_device(rbuf[slot].data_ptr(), rows * W * 3, precision=args.precision, rng=args.rng,
                            device=local, row_offset=rank, row_stride=world, stream=rs.cuda_stream, trace=args.trace)
        e1.record(rs)
        if timed:
            rend.append((e0, e1))
        if isolated:
            single["ev"] = (e0, e1)
        ready = e1
        if world > 1:  # the single RCCL collective + un-permute on rank 0
            stream.wait_event(e1)
            fr = frames[slot] if lead else None
            if lead and copied[slot] is not None:
                stream.wait_event(copied[slot])  # frame buffer `slot` was copied out NB frames ago
            shard.gather_frame(rbuf[slot], H, dist, rank, world, out=fr, host=args.backend == "gloo")
            ready = torch.cuda.Event()
            ready.record(stream)
            freed[slot] = ready
        else:
            freed[slot] = e1
        if lead and not args.kernel_only:
            cs = rs if copy_on_render else copy_stream
            if not copy_on_render:
                cs.wait_event(ready)
            c0, c1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            src = frames[slot]
            with torch.cuda.stream(cs):
                c0.record(cs)
                host[slot].view(-1).copy_(src.view(-1)[: H * W * 3], non_blocking=True)
                c1.record(cs)
            copied[slot] = c1
            if world == 1:
                freed[slot] = c1
            if timed:
                cev.append((c0, c1))

    first_frame = None
    for k in range(args.warmup):
        if k == args.warmup - 1 and k > 0:
            torch.cuda.synchronize()  # the last warm-up frame alone on the GPU: the single-frame latency
        step(k, False, isolated=k == args.warmup - 1 and k > 0)
        if k == 0:
            torch.cuda.synchronize()
            first_frame = time.perf_counter() - t_first0
    torch.cuda.synchronize()
    single_ms = single["ev"][0].elapsed_time(single["ev"][1]) if single else None
    jit_before = nrt.jit_stats()  # the first render of the scene in a world mode built its kernel (warm-up)
    if world > 1:
        dist.barrier()
    t0 = time.perf_counter()
    for k in range(args.steps):
        step(args.warmup + k, True)
    torch.cuda.synchronize()  # every frame's device-to-host copy has landed
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    # the render's device time per frame: from the first timed render's start to the last render end, over
    # the frames (with --pipeline > 1 consecutive renders overlap at their ends, and a frame may even end
    # before the one launched just ahead of it on the other stream, so neither one launch's own begin..end
    # nor the gap between successive end events is the time a frame costs)
    if rend:
        kern_ms = max(rend[0][0].elapsed_time(e1) for _, e1 in rend) / len(rend)
    else:
        kern_ms = single_ms if single_ms is not None else elapsed / max(args.steps, 1) * 1e3
    d2h_ms = sum(a.elapsed_time(b) for a, b in cev) / max(len(cev), 1) if cev else 0.0
    jit_after = nrt.jit_stats()
    specialised = jit_after["launches"] - jit_before["launches"] >= args.steps
    mixed = False
    if world > 1:
        # max over ranks of the times; min and max over ranks of "timed on the scene-specialised kernel"
        # (the generic kernel renders the same bits, kernel.hpp fmad, but slower: a mix is reported)
        t = torch.tensor([elapsed, kern_ms, float(specialised), -float(specialised)], dtype=torch.float64,
                         device=dev if args.backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
        mixed = float(t[2]) != -float(t[3])
    variant = kernel_variant_of(jit_before, jit_after, args.steps, mixed)
    if lead:
        last = host[(args.warmup + args.steps - 1) % NB].numpy()
        frame_sha = None if args.kernel_only else hashlib.sha256(last.tobytes()).hexdigest()
        report(args, nrt, scene, n_gpus=world, rows=rows, elapsed=elapsed, kern_ms=kern_ms, d2h_ms=d2h_ms,
               timings_s={"runtime_init": round(t_init, 4), "scene_load_and_bvh": round(t_load, 4),
                          "upload": round(t_upload, 4), "jit_compile": jit_after["compile_s"],
                          "first_frame": None if first_frame is None else round(first_frame, 4)},
               frame_sha=frame_sha, jit_before=jit_before, jit_after=jit_after, kernel_variant=variant,
               parallelism=f"rows interleaved over {world} GPU(s), one RCCL gather to rank 0",
               extra=dict({"pipeline": {"frames_in_flight": D, "single_frame_render_ms":
                                        None if single_ms is None else round(single_ms, 3),
                                        "note": "kernel_ms = device time from the first timed render's start to the "
                                                "last render's end, per frame; single_frame_render_ms "
                                                "= one render alone on an idle GPU (the last warm-up frame, after a "
                                                "synchronize: launch latency and clock ramp included)"}},
                          **({"multi_gpu": {"path": "ranks", "backend": args.backend}} if world > 1 else {})))
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
