#!/usr/bin/env python3
"""Summarise a scripts/profile.sh run (gpurun_out/prof) into profiles/<tag>_*.

Writes
  profiles/<tag>_kernel_stats.csv   rocprofv3 --kernel-trace --stats summary (copied)
  profiles/<tag>_pmc.md             per-launch PMC averages for the trace kernel
  profiles/pmc_traffic.json         HBM bytes per trace launch, read by bench.py

HBM traffic per launch follows MI355X_MICROARCH.md §HBM: FETCH_SIZE and WRITE_SIZE are
in KiB, from separate passes; on gfx950 FETCH_SIZE reports half the bytes of a wide
coalesced read, so it is doubled (an upper estimate for this kernel's narrow loads).
"""
import csv
import json
import os
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(REPO, "gpurun_out", os.environ.get("PROF_DIR", "prof"))
KERNEL = os.environ.get("PROF_KERNEL", "trace_pool")   # the timed variant (COUNT = false)


def per_launch(path, kernel=KERNEL):
    vals = {}
    meta = {}
    for r in csv.DictReader(open(path)):
        if kernel not in r["Kernel_Name"] or "true> >" in r["Kernel_Name"]:
            continue
        vals.setdefault(r["Counter_Name"], []).append(float(r["Counter_Value"]))
        meta = {k: r[k] for k in ("Grid_Size", "Workgroup_Size", "VGPR_Count", "SGPR_Count", "Scratch_Size",
                                  "LDS_Block_Size")}
        meta["duration_ns"] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
    return {k: statistics.mean(v) for k, v in vals.items()}, meta


def main():
    tag = sys.argv[1] if len(sys.argv) > 1 else "r01"
    config = sys.argv[2] if len(sys.argv) > 2 else "1200x800x500 depth 50 random scene"
    out = os.path.join(REPO, "profiles")
    os.makedirs(out, exist_ok=True)
    stats = os.path.join(PROF, "kt", "kt_kernel_stats.csv")
    shutil.copy(stats, os.path.join(out, f"{tag}_kernel_stats.csv"))
    avg_ns = None
    for r in csv.DictReader(open(stats)):
        if KERNEL in r["Name"] and "true> >" not in r["Name"]:
            avg_ns = float(r["AverageNs"])
    counters, meta = {}, {}
    for sub in ("fetch", "write", "sq"):
        p = os.path.join(PROF, sub, f"{sub}_counter_collection.csv")
        if os.path.exists(p):
            c, m = per_launch(p)
            counters.update(c)
            meta = meta or m
    fetch_b = counters.get("FETCH_SIZE", 0.0) * 1024
    write_b = counters.get("WRITE_SIZE", 0.0) * 1024
    traffic = 2 * fetch_b + write_b
    lines = [f"# PMC summary `{tag}` — {KERNEL}, {config}", "",
             f"kernel-trace average duration: {avg_ns / 1e6:.3f} ms" if avg_ns else "", "",
             "| counter | per launch |", "|---|---|"]
    for k in sorted(counters):
        lines.append(f"| {k} | {counters[k]:.6g} |")
    lines += ["", f"dispatch: {meta}", "",
              f"HBM traffic per launch = 2*FETCH_SIZE + WRITE_SIZE = {traffic / 1e6:.1f} MB "
              f"(fetch {fetch_b / 1e6:.2f} MB raw, write {write_b / 1e6:.1f} MB)"]
    if "GRBM_GUI_ACTIVE" in counters and avg_ns:
        lines.append(f"effective clock ~ GRBM_GUI_ACTIVE/8/t = {counters['GRBM_GUI_ACTIVE'] / 8 / (avg_ns * 1e-9) / 1e9:.2f} GHz")
    valu_busy = None
    if "SQ_ACTIVE_INST_VALU" in counters and counters.get("GRBM_GUI_ACTIVE"):
        # quad-cycles of VALU issue summed over waves, x4 -> cycles, over the SIMD-cycles of
        # the launch (1024 SIMDs x GRBM_GUI_ACTIVE / 8 XCDs): ~1 means VALU-issue bound
        valu_busy = 4.0 * counters["SQ_ACTIVE_INST_VALU"] / (1024.0 * counters["GRBM_GUI_ACTIVE"] / 8.0)
        lines.append(f"VALU issue busy ~ 4*SQ_ACTIVE_INST_VALU / (1024 SIMDs * GRBM_GUI_ACTIVE/8) = {valu_busy:.3f}")
    if "SQ_THREAD_CYCLES_VALU" in counters and "SQ_ACTIVE_INST_VALU" in counters:
        lines.append(f"VALU lane utilisation ~ SQ_THREAD_CYCLES_VALU / (64*SQ_ACTIVE_INST_VALU) = "
                     f"{counters['SQ_THREAD_CYCLES_VALU'] / (64 * counters['SQ_ACTIVE_INST_VALU']):.3f}")
    open(os.path.join(out, f"{tag}_pmc.md"), "w").write("\n".join(lines) + "\n")
    workload = [int(x) for x in os.environ.get("PROF_WORKLOAD", "0,1200,800,500,50,1").split(",")]
    schedule = 1 if KERNEL == "trace_pool" else 0
    path = os.path.join(out, "pmc_traffic.json")
    entries = []
    if os.path.exists(path):
        entries = [e for e in json.load(open(path)).get("entries", [])
                   if not (e.get("workload") == workload and e.get("schedule") == schedule)]
    entries.append({"tag": tag, "config": config, "workload": workload, "kernel": KERNEL, "schedule": schedule,
                    "hbm_bytes_per_launch": traffic,
                    "fetch_size_kib": counters.get("FETCH_SIZE"), "write_size_kib": counters.get("WRITE_SIZE"),
                    "kernel_avg_ns": avg_ns, "valu_busy": valu_busy})
    json.dump({"note": "HBM bytes per trace-kernel launch (2*FETCH_SIZE + WRITE_SIZE, KiB*1024), "
                       "from scripts/profile.sh + scripts/prof_summary.py; bench.py matches workload "
                       "[scene, W, H, spp, depth, n_gpus] and schedule",
               "entries": entries}, open(path, "w"), indent=1)
    print("\n".join(lines))


if __name__ == "__main__":
    main()
