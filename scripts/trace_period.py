"""Render-kernel timing from a rocprofv3 kernel trace (run_kernel_trace.csv), for pipelined runs.

usage: python scripts/trace_period.py <rocprofv3 -d dir or run_kernel_trace.csv> [--json out.json]

With bench.py --pipeline 1 consecutive frames' render launches overlap at their ends (frame k+1's
workgroups start on the SIMDs frame k's last paths leave idle), so one dispatch's begin..end also
counts the other frame's tail and rocprofv3's AverageNs exceeds the time a frame costs.  This prints,
per render-kernel name: dispatches, the mean begin..end duration (what --stats averages), the
steady-state period = (last end - first start) / n over the dispatches after the first two (warm-up /
module load), which is what bench.py's roofline.kernel_ms measures with HIP events, and
the overlap between consecutive dispatches.
"""
import argparse
import csv
import glob
import json
import os
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("src")
    ap.add_argument("--json")
    ap.add_argument("--skip", type=int, default=None,
                    help="leading dispatches left out of the period (the warm-up frames; default: the `warmup` of the "
                         "bench line next to the trace, bench_trace.json, else 2)")
    a = ap.parse_args()
    path = a.src
    if a.skip is None:
        a.skip = 2
        bt = os.path.join(os.path.dirname(os.path.normpath(path if os.path.isdir(path) else os.path.dirname(path))),
                          "bench_trace.json")
        if os.path.exists(bt):
            try:
                a.skip = int(json.loads(open(bt).read().strip().splitlines()[-1])["warmup"])
            except (ValueError, KeyError, IndexError):
                pass
    if os.path.isdir(path):
        path = next(iter(glob.glob(os.path.join(path, "**", "*kernel_trace.csv"), recursive=True)), None)
        if path is None:
            sys.exit("no *kernel_trace.csv")
    rows = {}
    with open(path) as fh:
        for r in csv.DictReader(fh):
            name = r["Kernel_Name"]
            if "render_kernel" not in name:
                continue
            rows.setdefault(name, []).append((int(r["Start_Timestamp"]), int(r["End_Timestamp"])))
    out = {}
    for name, d in rows.items():
        d.sort(key=lambda x: x[1])
        dur = [e - s for s, e in d]
        steady = d[a.skip:]
        # first start to last end over the steady dispatches, per dispatch (consecutive dispatches
        # overlap, and one may even end before the one launched just ahead of it: end-to-end gaps
        # alone are biased); None with fewer than two (a run of 1-2 timed frames: the warm-up's host
        # synchronize would sit inside the span)
        period = ((max(e for _, e in steady) - min(s for s, _ in steady)) / len(steady)) if len(steady) >= 2 else None
        overlap = [max(0, d[i][1] - d[i + 1][0]) for i in range(len(d) - 1)]
        out[name] = {"dispatches": len(d), "mean_duration_ns": sum(dur) / len(dur),
                     "steady_period_ns": period, "steady_dispatches": len(steady),
                     "mean_overlap_ns": sum(overlap) / len(overlap) if overlap else 0.0,
                     "source": os.path.relpath(path)}
    print(json.dumps(out, indent=1))
    if a.json:
        with open(a.json, "w") as fh:
            json.dump(out, fh, indent=1)


if __name__ == "__main__":
    main()
