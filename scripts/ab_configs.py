"""A/B timing of library builds and kernel knobs on one GPU box (alternating runs).

usage: python scripts/ab_configs.py --reps 2 --out gpurun_out/ab.jsonl \
           --lib base=nr-ray-tracer_amd/ab/base/libnrt.so --lib new=nr-ray-tracer_amd/nrt/libnrt.so \
           --env w5="NRT_JIT_DEFS=-DNRT_WBVH_WAVES=5" \
           --cfg c4="--scene scenes/utah-teapot-scene.json" --cfg c5=""
Every (cfg, lib, env) combination runs `bench.py --steps S --warmup 1 --no-cpu-baseline <cfg>` as a
child process (own timeout), repeated --reps times in alternating order; one JSON line per run
goes to --out and a summary (best kernel ms per combination) to stdout.

A run is INVALID when its kernel variant is not the one the configuration's first arm ran, or when
a scene-specialised build failed (bench.py's "kernel_variant" then names the generic fallback): the
arm would time another kernel than the one it names.  Invalid runs are marked ("valid": false), left
out of the summary, and make the script exit with status 3 at the end.
"""
import argparse
import json
import os
import shlex
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def kv(s):
    k, _, v = s.partition("=")
    return k, v


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--lib", action="append", type=kv, default=[])
    ap.add_argument("--env", action="append", type=kv, default=[])
    ap.add_argument("--cfg", action="append", type=kv, default=[])
    ap.add_argument("--arm", action="append", type=kv, default=[],
                    help="NAME=LIBPATH::ENV ... : one (library, environment) pair, instead of the --lib x --env product")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--timeout", type=int, default=120)
    ap.add_argument("--out", default="gpurun_out/ab.jsonl")
    a = ap.parse_args()
    libs = a.lib or [("cur", os.path.join(ROOT, "nr-ray-tracer_amd", "nrt", "libnrt.so"))]
    envs = a.env or [("-", "")]
    cfgs = a.cfg or [("c5", "")]
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    best = {}
    base_variant = {}  # cfg -> kernel_variant of its first run
    invalid = []
    with open(a.out, "a") as fh:
        for rep in range(a.reps):
            for cname, cargs in cfgs:
                combos = [(l, e) for l in libs for e in envs]
                if a.arm:
                    combos = []
                    for name, spec in a.arm:
                        lp, _, es = spec.partition("::")
                        combos.append(((name, lp or libs[0][1]), ("-", es)))
                if rep % 2:
                    combos.reverse()
                for (lname, lpath), (ename, estr) in combos:
                    env = dict(os.environ, NRT_LIB=os.path.abspath(lpath))
                    for tok in shlex.split(estr):
                        k, _, v = tok.partition("=")
                        env[k] = v
                    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--steps", str(a.steps), "--warmup", "1",
                           "--no-cpu-baseline", *shlex.split(cargs)]
                    t0 = time.time()
                    r = subprocess.run(cmd, capture_output=True, text=True, timeout=a.timeout, env=env, cwd=ROOT)
                    if r.returncode != 0:
                        print(f"FAIL {cname} {lname} {ename} rc={r.returncode}\n{r.stderr[-1500:]}", flush=True)
                        sys.exit(1)
                    d = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
                    variant = str(d.get("kernel_variant"))
                    base = base_variant.setdefault(cname, variant)
                    valid = variant == base and "FAILED" not in variant and "MIXED" not in variant
                    rec = {"cfg": cname, "lib": lname, "env": ename, "rep": rep, "value": d["value"],
                           "kernel_ms": d["timings_ms"]["kernel_device_only"], "frame_sha256": d["frame_sha256"],
                           "kernel_variant": variant, "valid": valid, "wall_s": round(time.time() - t0, 1)}
                    fh.write(json.dumps(rec) + "\n")
                    fh.flush()
                    print(f"{cname:8s} {lname:8s} {ename:10s} {d['value']:10.1f} Msamples/s "
                          f"{rec['kernel_ms']:9.3f} ms  {str(d['frame_sha256'])[:12]}  {variant}"
                          + ("" if valid else "  INVALID"), flush=True)
                    key = (cname, lname, ename)
                    if valid:
                        best[key] = min(best.get(key, 1e30), rec["kernel_ms"])
                    else:
                        invalid.append(key)
    print("best kernel ms:")
    for (c, l, e), ms in best.items():
        print(f"  {c:8s} {l:8s} {e:10s} {ms:9.3f}")
    if invalid:
        print(f"INVALID arms (kernel variant differs from the first arm's or a build failed): "
              f"{sorted(set(invalid))}", flush=True)
        sys.exit(3)


if __name__ == "__main__":
    main()
