"""Copy profile runs (scripts/profile.sh <tag>_<variant> ...) from gpurun_out/ into profiles/.

usage: python scripts/publish_profiles.py <tag> [--as r02] [--bench <tag>_bench_default.json]

For every gpurun_out/prof_<tag>_<variant>/ directory writes
  profiles/<as>_<variant>_kernel_stats.csv  (rocprofv3 --kernel-trace --stats summary)
  profiles/<as>_<variant>_pmc.json          (scripts/pmc_summary.py over the PMC passes)
and profiles/pmc_summary.json: one entry per variant, keyed by the exact bench configuration
of that run (scene, width, height, spp, precision, rng, trace, n_gpus, read from the bench line
the kernel-trace run printed), which bench.py looks up for its roofline block.
"""
import argparse
import glob
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
KEY = ("scene", "width", "height", "spp", "precision", "rng", "trace")
KEEP = ("kernel", "avg_ns", "calls", "hbm_bytes_per_launch", "hbm_fetch_bytes", "hbm_write_bytes",
        "valu_lane_utilization", "valu_insts_per_wave", "valu_issue_frac", "clock_mhz", "wait_inst_frac",
        "wait_any_frac", "lds_bank_conflict_frac", "tcc_hit_rate", "tcp_to_tcc_frac", "valu_busy_est",
        "valu_cycles_per_inst_est", "valu_mix")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--as", dest="name", default="r02")
    a = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    entries = []
    dirs = sorted(glob.glob(os.path.join(ROOT, "gpurun_out", f"prof_{a.tag}_*")))
    if not dirs:
        sys.exit(f"no gpurun_out/prof_{a.tag}_* directories")
    for src in dirs:
        v = os.path.basename(src)[len(f"prof_{a.tag}_"):]
        stats = os.path.join(src, "trace", "run_kernel_stats.csv")
        if not os.path.exists(stats):
            stats = next(iter(glob.glob(os.path.join(src, "trace", "**", "*kernel_stats.csv"), recursive=True)), None)
        if stats is None:
            print(f"skip {v}: no kernel stats")
            continue
        shutil.copy(stats, os.path.join(prof, f"{a.name}_{v}_kernel_stats.csv"))
        tp = os.path.join(src, "trace_period.json")  # scripts/trace_period.py (pipelined runs)
        if not os.path.exists(tp):
            subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "trace_period.py"), os.path.join(src, "trace"),
                            "--json", tp], check=False, capture_output=True)
        period = None
        if os.path.exists(tp):
            with open(tp) as fh:
                period = next(iter(json.load(fh).values()), {}).get("steady_period_ns")
        pmc_json = os.path.join(prof, f"{a.name}_{v}_pmc.json")
        subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_summary.py"), src, "--json", pmc_json] +
                       (["--period-ns", str(period)] if period else []), check=True, capture_output=True)
        with open(pmc_json) as fh:
            d = json.load(fh)
        with open(os.path.join(src, "bench_trace.json")) as fh:
            bench = json.loads(fh.read().strip().splitlines()[-1])
        e = {k: bench["config"][k] for k in KEY}
        e["n_gpus"] = bench["n_gpus"]
        e["variant"] = v
        e.update({k: d.get(k) for k in KEEP})
        e["bench_kernel_ms"] = bench["roofline"]["kernel_ms"]
        if os.path.exists(tp):
            shutil.copy(tp, os.path.join(prof, f"{a.name}_{v}_trace_period.json"))
            with open(tp) as fh:
                per = next(iter(json.load(fh).values()), {})
            e["steady_period_ns"] = per.get("steady_period_ns")
            e["mean_overlap_ns"] = per.get("mean_overlap_ns")
        e["source"] = (f"profiles/{a.name}_{v}_pmc.json + {a.name}_{v}_kernel_stats.csv (rocprofv3 --kernel-trace "
                       f"--stats, then --pmc, one counter group per pass; FETCH_SIZE x2 per MI355X_MICROARCH.md; "
                       f"valu_issue_frac in 2-cycle wave64 slots)")
        entries.append(e)
    # merge: entries of other configurations (earlier rounds' profiles) stay until re-profiled
    summ = os.path.join(prof, "pmc_summary.json")
    old = []
    if os.path.exists(summ):
        with open(summ) as fh:
            old = json.load(fh).get("entries", [])
    keyof = lambda e: tuple(e.get(k) for k in KEY + ("n_gpus",))  # noqa: E731
    new_keys = {keyof(e) for e in entries}
    merged = [e for e in old if keyof(e) not in new_keys] + entries
    with open(summ, "w") as fh:
        fh.write(json.dumps({"round": a.name, "entries": merged}, indent=1) + "\n")
    print(json.dumps(entries, indent=1))


if __name__ == "__main__":
    main()
