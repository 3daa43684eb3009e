"""Summarise rocprofv3 kernel-trace + PMC CSVs of one profile run (scripts/profile.sh).

usage: python scripts/pmc_summary.py gpurun_out/prof_<tag> [--kernel render_kernel] [--json out.json]
HBM bytes follow MI355X_MICROARCH.md §HBM: FETCH_SIZE (KiB) reads half of a wide
coalesced stream on gfx950, so it is doubled; WRITE_SIZE (KiB) is exact for
16-B-per-lane stores and uncalibrated for the 4-B stores this kernel issues.
"""
import argparse
import collections
import csv
import glob
import json
import os


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("dir")
    ap.add_argument("--kernel", default="render_kernel")
    ap.add_argument("--json")
    ap.add_argument("--ubench", default=os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))),
                                                     "profiles", "r02_ubench_valu_cost.jsonl"),
                    help="scripts/ubench/valu_cost output: per-class issue cost at 8 waves per SIMD")
    ap.add_argument("--period-ns", type=float, default=None,
                    help="the kernel's steady period from the same command's trace (scripts/trace_period.py): the "
                         "time base of clock_mhz.  rocprofv3 --stats AverageNs is no time base with frames in flight "
                         "(a dispatch's begin..end spans its wait behind the ones ahead), so without it no clock is "
                         "reported")
    a = ap.parse_args()
    out = {}
    st = glob.glob(os.path.join(a.dir, "trace", "**", "*kernel_stats.csv"), recursive=True)
    if st:
        for r in csv.DictReader(open(st[0])):
            if a.kernel in r["Name"]:
                out["kernel"] = r["Name"]
                out["calls"] = int(r["Calls"])
                out["avg_ns"] = float(r["AverageNs"])
    agg = collections.defaultdict(float)
    disp = collections.defaultdict(set)
    grbm_ns = []  # the GRBM pass's own dispatch durations (counter passes serialise dispatches)
    by_disp = collections.defaultdict(float)
    files = glob.glob(os.path.join(a.dir, "pmc*", "**", "*counter_collection.csv"), recursive=True)
    if not files:  # a single PMC pass's output directory
        files = glob.glob(os.path.join(a.dir, "**", "*counter_collection.csv"), recursive=True)
    for f in files:
        for r in csv.DictReader(open(f)):
            if a.kernel in r.get("Kernel_Name", ""):
                agg[r["Counter_Name"]] += float(r["Counter_Value"])
                disp[r["Counter_Name"]].add(r.get("Dispatch_Id", ""))
                by_disp[(r["Counter_Name"], f, r.get("Dispatch_Id", ""))] += float(r["Counter_Value"])
                if r["Counter_Name"] == "GRBM_GUI_ACTIVE" and r.get("Start_Timestamp") and r.get("End_Timestamp"):
                    grbm_ns.append(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
    # per dispatch: the MEDIAN over the pass's dispatches (device-wide counters also count what else ran in
    # a dispatch's window: one of C5 f64's three profiled dispatches showed 196 MB of writes against 21.8 MB
    # for the other two, round 6); the mean stays beside it
    mean = {k: v / max(len(disp[k]), 1) for k, v in agg.items()}
    vals = collections.defaultdict(list)
    for (c, _, _), v in by_disp.items():
        vals[c].append(v)
    per = {c: sorted(v)[len(v) // 2] if len(v) % 2 else 0.5 * (sorted(v)[len(v) // 2 - 1] + sorted(v)[len(v) // 2])
           for c, v in vals.items()}
    out["per_dispatch"] = per
    out["per_dispatch_mean"] = mean
    out["per_dispatch_basis"] = "median over the PMC pass's dispatches of this kernel (per_dispatch_mean: the mean)"
    if "FETCH_SIZE" in per or "WRITE_SIZE" in per:
        fetch = per.get("FETCH_SIZE", 0.0) * 1024 * 2
        write = per.get("WRITE_SIZE", 0.0) * 1024
        out["hbm_bytes_per_launch"] = fetch + write
        out["hbm_fetch_bytes"] = fetch
        out["hbm_write_bytes"] = write
    if "SQ_INSTS_VALU" in per and "SQ_WAVES" in per:
        out["valu_insts_per_wave"] = per["SQ_INSTS_VALU"] / per["SQ_WAVES"]
    if "SQ_THREAD_CYCLES_VALU" in per and "SQ_ACTIVE_INST_VALU" in per and per["SQ_ACTIVE_INST_VALU"]:
        out["valu_lane_utilization"] = per["SQ_THREAD_CYCLES_VALU"] / (64.0 * per["SQ_ACTIVE_INST_VALU"])
    if "GRBM_GUI_ACTIVE" in per and "SQ_INSTS_VALU" in per and per["GRBM_GUI_ACTIVE"]:
        # GRBM_GUI_ACTIVE sums the busy cycles of the 8 XCDs.  A full-rate wave64 VALU
        # instruction occupies its SIMD-32 for 2 cycles when several waves share the SIMD
        # (MI355X_MICROARCH.md per-instruction constants, v_fma_f32), 1024 SIMDs.  Quarter-rate
        # and transcendental instructions hold the SIMD longer, so this is the issue fraction
        # counted in full-rate slots: a lower bound on how busy the vector pipe was.
        clk = per["GRBM_GUI_ACTIVE"] / 8.0  # busy cycles of one XCD per dispatch (PMC passes serialise dispatches)
        out["xcd_busy_cycles"] = clk
        if grbm_ns:
            out["pmc_dispatch_ns"] = sum(grbm_ns) / len(grbm_ns)
            out["clock_mhz"] = clk / (out["pmc_dispatch_ns"] * 1e-9) / 1e6
            out["clock_basis"] = ("GRBM_GUI_ACTIVE / 8 over the same PMC pass's dispatch duration (its Start/End "
                                  "timestamps; counter passes run dispatches one at a time)")
        elif a.period_ns:
            out["clock_mhz"] = clk / (a.period_ns * 1e-9) / 1e6
            out["clock_basis"] = "GRBM_GUI_ACTIVE / 8 over the trace's steady period (--period-ns)"
        out["valu_issue_frac"] = per["SQ_INSTS_VALU"] * 2.0 / (1024.0 * clk)
    if "SQ_WAIT_INST_ANY" in per and per.get("SQ_WAVE_CYCLES"):
        out["wait_inst_frac"] = per["SQ_WAIT_INST_ANY"] / per["SQ_WAVE_CYCLES"]
        out["wait_any_frac"] = per.get("SQ_WAIT_ANY", 0.0) / per["SQ_WAVE_CYCLES"]
    if per.get("SQ_LDS_IDX_ACTIVE"):
        out["lds_bank_conflict_frac"] = per.get("SQ_LDS_BANK_CONFLICT", 0.0) / per["SQ_LDS_IDX_ACTIVE"]
    if per.get("TCC_HIT_sum", 0.0) + per.get("TCC_MISS_sum", 0.0) > 0:
        out["tcc_hit_rate"] = per["TCC_HIT_sum"] / (per["TCC_HIT_sum"] + per["TCC_MISS_sum"])
    if per.get("TCP_TOTAL_CACHE_ACCESSES_sum"):
        # vector L1 requests that went on to L2 per L1 access (1 - L1 hit rate, approximately)
        out["tcp_to_tcc_frac"] = per.get("TCP_TCC_READ_REQ_sum", 0.0) / per["TCP_TOTAL_CACHE_ACCESSES_sum"]
    # VALU busy estimate: each instruction class priced at its measured wall-clock issue cost per
    # SIMD with 8 waves per SIMD on every CU (scripts/ubench/valu_cost.hip), over the SIMD cycles
    # of the dispatch.  Unclassified VALU (compares, selects, moves, bit ops) at the v_add_f32 cost.
    classes = {"SQ_INSTS_VALU_ADD_F32": "v_add_f32", "SQ_INSTS_VALU_MUL_F32": "v_mul_f32",
               "SQ_INSTS_VALU_FMA_F32": "v_fma_f32", "SQ_INSTS_VALU_TRANS_F32": "v_exp_f32",
               "SQ_INSTS_VALU_INT32": "v_xor_b32", "SQ_INSTS_VALU_INT64": "v_mad_u64_u32",
               "SQ_INSTS_VALU_CVT": "v_cvt_f32_u32", "SQ_INSTS_VALU_FMA_F64": "v_fma_f64",
               "SQ_INSTS_VALU_ADD_F64": "v_mul_f64", "SQ_INSTS_VALU_MUL_F64": "v_mul_f64",
               "SQ_INSTS_VALU_TRANS_F64": "v_exp_f32"}
    if os.path.exists(a.ubench) and out.get("xcd_busy_cycles") and "SQ_INSTS_VALU_FMA_F32" in per and "SQ_INSTS_VALU" in per:
        cyc = {}
        for line in open(a.ubench):
            d = json.loads(line)
            if d.get("waves_per_simd") == 8:
                cyc[d["op"]] = d["clock_mhz"] * 1e6 / d["wall_wave_insts_per_s_per_simd"]
        if all(v in cyc for v in classes.values()) and "v_add_f32" in cyc:
            busy = 0.0
            known = 0.0
            mix = {}
            for c, op in classes.items():
                n = per.get(c, 0.0)
                busy += n * cyc[op]
                known += n
                mix[c.replace("SQ_INSTS_VALU_", "")] = n / per["SQ_INSTS_VALU"]
            other = max(per["SQ_INSTS_VALU"] - known, 0.0)
            busy += other * cyc["v_add_f32"]
            mix["OTHER"] = other / per["SQ_INSTS_VALU"]
            simd_cycles = 1024.0 * out["xcd_busy_cycles"]  # (no time base needed: cycles, not seconds)
            out["valu_mix"] = mix
            out["valu_cycles_per_inst_est"] = busy / per["SQ_INSTS_VALU"]
            out["valu_busy_est"] = busy / simd_cycles
            out["valu_busy_source"] = a.ubench
    text = json.dumps(out, indent=1, sort_keys=True)
    print(text)
    if a.json:
        with open(a.json, "w") as fh:
            fh.write(text + "\n")


if __name__ == "__main__":
    main()
