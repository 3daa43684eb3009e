"""Alternating bench runs of several arms of one config (round-robin, so box drift hits every arm alike).

usage: python scripts/ab_arms.py <tag> <reps> --arm NAME='VAR=value;VAR2=value two' [--arm ...] -- <bench args...>
An arm's environment assignments are separated by ';' (values may hold spaces, e.g. NRT_JIT_DEFS);
arm "A" with no assignment is always run first.  Each run is `bench.py --no-cpu-baseline <bench args>`
under a 300-s limit; the first failing run stops the script (no retries).  Prints one line per run and
a per-arm summary (min / median of the kernel ms and the value), writes gpurun_out/<tag>_ab.jsonl.
"""
import json
import os
import statistics
import subprocess
import sys


def main():
    argv = sys.argv[1:]
    tag, reps = argv[0], int(argv[1])
    argv = argv[2:]
    arms = [("A", {})]
    while argv and argv[0] == "--arm":
        name, _, spec = argv[1].partition("=")
        env = {}
        for a in spec.split(";"):
            if a:
                k, _, v = a.partition("=")
                env[k] = v
        arms.append((name, env))
        argv = argv[2:]
    if argv and argv[0] == "--":
        argv = argv[1:]
    os.makedirs("gpurun_out", exist_ok=True)
    rows = []
    for r in range(reps):
        for name, env in arms:
            e = dict(os.environ)
            e.update(env)
            p = subprocess.run(["timeout", "-k", "10", "300", sys.executable, "bench.py", "--no-cpu-baseline", *argv],
                               env=e, capture_output=True, text=True)
            if p.returncode != 0:
                sys.stderr.write(p.stderr[-3000:])
                sys.exit(f"{tag} arm {name} rep {r}: exit {p.returncode}")
            d = json.loads(p.stdout.strip().splitlines()[-1])
            row = {"tag": tag, "arm": name, "env": env, "rep": r, "value": d["value"], "ms_per_step": d["ms_per_step"],
                   "kernel_ms": d["roofline"].get("kernel_ms"), "sha": (d.get("frame_sha256") or "")[:12],
                   "variant": d.get("kernel_variant")}
            rows.append(row)
            print(json.dumps(row), flush=True)
    with open(f"gpurun_out/{tag}_ab.jsonl", "w") as fh:
        for row in rows:
            fh.write(json.dumps(row) + "\n")
    for name, _ in arms:
        v = [x["value"] for x in rows if x["arm"] == name]
        k = [x["kernel_ms"] for x in rows if x["arm"] == name and x["kernel_ms"]]
        print(f"{tag} {name}: value min {min(v):.1f} med {statistics.median(v):.1f} max {max(v):.1f}; "
              f"kernel ms min {min(k) if k else 0:.3f} med {statistics.median(k) if k else 0:.3f}", flush=True)


if __name__ == "__main__":
    main()
