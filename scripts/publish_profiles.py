"""Copy one round-profile run (scripts/round_profile.sh <tag>) from gpurun_out/ into profiles/.

usage: python scripts/publish_profiles.py <tag> [--as r01]

Writes profiles/<as>_<variant>_kernel_stats.csv (rocprofv3 --kernel-trace --stats summary),
profiles/<as>_<variant>_pmc.json (scripts/pmc_summary.py over the PMC passes),
profiles/<as>_bench_default.json (the default bench line of the same call) and
profiles/pmc_summary.json, the per-variant figures bench.py quotes in its roofline block.
"""
import argparse
import json
import os
import shutil
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
VARIANTS = ("f32_philox", "f64_chacha8")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tag")
    ap.add_argument("--as", dest="name", default="r01")
    a = ap.parse_args()
    prof = os.path.join(ROOT, "profiles")
    summary = {}
    for v in VARIANTS:
        src = os.path.join(ROOT, "gpurun_out", f"prof_{a.tag}_{v}")
        if not os.path.isdir(src):
            sys.exit(f"missing {src}")
        shutil.copy(os.path.join(src, "trace", "run_kernel_stats.csv"),
                    os.path.join(prof, f"{a.name}_{v}_kernel_stats.csv"))
        pmc_json = os.path.join(prof, f"{a.name}_{v}_pmc.json")
        subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "pmc_summary.py"), src, "--json", pmc_json],
                       check=True, capture_output=True)
        with open(pmc_json) as fh:
            d = json.load(fh)
        keep = ("kernel", "avg_ns", "hbm_bytes_per_launch", "hbm_fetch_bytes", "hbm_write_bytes",
                "valu_lane_utilization", "valu_insts_per_wave", "valu_issue_frac", "clock_mhz")
        summary[v] = {k: d.get(k) for k in keep}
        summary[v]["source"] = (f"profiles/{a.name}_{v}_pmc.json (rocprofv3 --pmc, one counter group per pass; "
                                f"FETCH_SIZE x2 per MI355X_MICROARCH.md; valu_issue_frac in 2-cycle wave64 slots)")
    bench = os.path.join(ROOT, "gpurun_out", f"{a.tag}_bench_default.json")
    if os.path.exists(bench):
        shutil.copy(bench, os.path.join(prof, f"{a.name}_bench_default.json"))
    with open(os.path.join(prof, "pmc_summary.json"), "w") as fh:
        fh.write(json.dumps(summary, indent=1) + "\n")
    print(json.dumps(summary, indent=1))


if __name__ == "__main__":
    main()
