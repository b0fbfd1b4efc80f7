#!/usr/bin/env python3
"""Summarise rocprofv3 runs into profiles/ (round 2 format).

  python scripts/pmc_r02.py calib <gpurun_out dir> <tag>
      scripts/calib_r02.sh output -> the VALU calibration block of profiles/pmc.json
      and profiles/<tag>_valu_calib.md
  python scripts/pmc_r02.py bench <gpurun_out dir> <tag> <scene,W,H,spp,depth,n_gpus,schedule> [note]
      scripts/profile_r02.sh output -> one entry of profiles/pmc.json (keyed by the
      source hash of this tree and the workload), profiles/<tag>_pmc.md and
      profiles/<tag>_kernel_stats.csv

Counter reading (MI355X_MICROARCH.md §HBM, §rocprofv3 PMC slots, §Per-instruction cycle
constants): SQ_* cycle counters count quad-cycles; GRBM_GUI_ACTIVE is summed over the 8
XCDs, so the clock the chip held = GRBM_GUI_ACTIVE / 8 / kernel time; FETCH_SIZE and
WRITE_SIZE are KiB, and on gfx950 FETCH_SIZE reports half the bytes of wide coalesced
reads, so DRAM bytes = 2 x FETCH_SIZE + WRITE_SIZE (an upper estimate for this kernel's
narrower loads; the kernel reads almost nothing from DRAM either way).
"""
import collections
import csv
import glob
import json
import os
import re
import shutil
import statistics
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
OUT_JSON = os.path.join(REPO, "profiles", "pmc.json")
N_SIMDS = 1024

# trace-kernel VALU classes (rocprofv3 counter) -> the calibration kernel measuring its rate
CLASS_COUNTERS = {
    "f64_add": "SQ_INSTS_VALU_ADD_F64", "f64_mul": "SQ_INSTS_VALU_MUL_F64", "f64_fma": "SQ_INSTS_VALU_FMA_F64",
    "f64_trans": "SQ_INSTS_VALU_TRANS_F64", "f32_add": "SQ_INSTS_VALU_ADD_F32", "f32_mul": "SQ_INSTS_VALU_MUL_F32",
    "f32_fma": "SQ_INSTS_VALU_FMA_F32", "f32_trans": "SQ_INSTS_VALU_TRANS_F32", "int32": "SQ_INSTS_VALU_INT32",
    "int64": "SQ_INSTS_VALU_INT64", "cvt": "SQ_INSTS_VALU_CVT"}
CLASS_PROXY = {"f64_add": ["f64_add"], "f64_mul": ["f64_mul"], "f64_fma": ["f64_fma"],
               "f64_trans": ["f64_rcp", "f64_sqrt"], "f32_add": ["f32_add"], "f32_mul": ["f32_add"],
               "f32_fma": ["f32_fma"], "f32_trans": ["f32_rcp"], "int32": ["i32_add"],
               "int64": ["lshl_b64"], "cvt": ["cvt_f64_u32"], "other": None}
# 'other' (instructions no class counter counts: moves, selects, compares, bit ops) is priced at
# the mean of the calibration ops that hit no class counter; bounds from their min / max
CALIB_OPS = ["f64_fma", "f64_add", "f64_mul", "f64_rcp", "f64_sqrt", "f32_fma", "f32_add", "f32_rcp", "i32_add",
             "i32_mul", "b32_xor", "cndmask", "mov_b32", "cndmask_vcc", "cmp_f64", "cmp_f32", "max_f64", "min_f32",
             "lshl_b64", "cvt_f64_u32", "bfe_u32", "pk_fma_f32", "max3_f32", "med3_f32", "and_b32", "or_b32",
             "lshl_b32", "lshr_b32", "alignbit_b32", "bitop3_b32", "mov_b64", "cmp_i32", "ldexp_f64", "div_scale_f64",
             "div_fmas_f64", "div_fixup_f64", "mad_u64_u32", "lshl_add_u64", "lshr_b64", "mbcnt_lo", "mul_hi_u32",
             "cvt_f32_f64", "cmp_class_f64", "sub_u32", "fmac_f64", "mul_f32", "rsq_f64", "cndmask_e32", "mix", "kmix_c2", "kmix_c4",
             "kmix_c3"]
# the MIX kernel's composition per accumulator-step (scripts/calib/valu_calib.hip): the model's
# prediction for it (sum of calibrated costs) against its measured rate validates additivity
MIX = {"f64_fma": 1, "f64_add": 1, "f32_fma": 2, "i32_add": 1, "b32_xor": 1, "mov_b32": 1, "cndmask": 1, "max3_f32": 1}


def read_counters(d, select):
    """{kernel key: {counter: mean per dispatch}, ...}, {kernel key: mean duration ns}."""
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    dur = {}
    kname = {}
    for f in sorted(glob.glob(os.path.join(d, "*", "*_counter_collection.csv"))):
        for r in csv.DictReader(open(f)):
            k = select(r["Kernel_Name"])
            if k is None:
                continue
            did = (f, r["Dispatch_Id"])
            per[(k, did)][r["Counter_Name"]] += float(r["Counter_Value"])
            dur[(k, did)] = int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
            kname[k] = r["Kernel_Name"]
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    durs = collections.defaultdict(list)
    for (k, did), cs in per.items():
        for c, v in cs.items():
            agg[k][c].append(v)
        durs[k].append(dur[(k, did)])
    return ({k: {c: statistics.mean(v) for c, v in cs.items()} for k, cs in agg.items()},
            {k: statistics.mean(v) for k, v in durs.items()}, kname)


def load():
    if os.path.exists(OUT_JSON):
        return json.load(open(OUT_JSON))
    return {"note": "rocprofv3 PMC per trace-kernel launch, keyed by source hash (__graft_entry__.source_hash) "
                    "and workload [scene, W, H, spp, depth, n_gpus, schedule]; calibration: VALU cycles per "
                    "wave-instruction per class at saturation (scripts/calib). Written by scripts/pmc_r02.py.",
            "calibration": None, "entries": []}


def calib(d, tag):
    ops = {i: n for i, n in enumerate(CALIB_OPS)}

    def sel(name):
        m = re.search(r"calib<(\d+), 8>", name)
        return ops[int(m.group(1))] if m else None

    counters, durs, _ = read_counters(d, sel)
    timing = [json.loads(l) for l in open(os.path.join(d, "timing.jsonl")) if l.strip()]
    lines = [f"# VALU issue calibration `{tag}` (scripts/calib/valu_calib.hip, MI355X)", "",
             "Saturated mode: 8 blocks x 256 threads per CU (8 waves per SIMD), 8 independent accumulators",
             "per lane, the class as one inline-asm instruction. cyc/inst (PMC) = 1024 SIMDs x",
             "(GRBM_GUI_ACTIVE/8) / SQ_INSTS_VALU; cyc/inst (timing) = SIMDs x hipEvent time x in-kernel",
             "clock / class instructions issued. 'one' = one wave per SIMD, 'lat' = one dependent chain.", "",
             "| op | cyc/inst PMC (sat) | clock GHz (PMC) | counters hit | ACTIVE_INST_VALU x4 / SIMD-cycles | "
             "cyc/inst timing sat | one | lat |", "|---|---|---|---|---|---|---|---|"]
    rates, unclassed, hit_map = {}, [], {}
    for op in CALIB_OPS:
        c = counters.get(op, {})
        t = {m: x for x in timing if x["op"] == op for m in [x["mode"]]}
        cyc = None
        if c.get("SQ_INSTS_VALU") and c.get("GRBM_GUI_ACTIVE"):
            cycles = c["GRBM_GUI_ACTIVE"] / 8.0
            cyc = N_SIMDS * cycles / c["SQ_INSTS_VALU"]
            clk = cycles / (durs[op] * 1e-9) / 1e9
            busy = 4.0 * c.get("SQ_ACTIVE_INST_VALU", 0.0) / (N_SIMDS * cycles)
        hits = [k[len("SQ_INSTS_VALU_"):] for k, v in c.items()
                if k.startswith("SQ_INSTS_VALU_") and v > 0.5 * c.get("SQ_INSTS_VALU", 1e30)]
        sat = t.get("sat", {}).get("cycles_per_inst_per_simd")
        rates[op] = cyc if cyc is not None else sat
        if c and not hits and op not in ("cndmask_vcc", "mix", "cndmask_e32", "kmix_c2", "kmix_c4", "kmix_c3"):   # pairs / mixes: not one op
            unclassed.append(op)
        hit_map[op] = hits
        lines.append(f"| {op} | {cyc if cyc is None else round(cyc, 3)} | "
                     f"{'' if cyc is None else round(clk, 3)} | {', '.join(hits)} | "
                     f"{'' if cyc is None else round(busy, 3)} | {sat if sat is None else round(sat, 3)} | "
                     f"{round(t['one']['cycles_per_inst_per_simd'], 3) if 'one' in t else ''} | "
                     f"{round(t['lat']['cycles_per_inst_per_simd'], 3) if 'lat' in t else ''} |")
    # the mix: predicted (sum of its instructions' calibrated costs) vs measured cycles per step
    mix_line = None
    if rates.get("mix") and all(rates.get(o) for o in MIX):
        n = sum(MIX.values())
        pred = sum(k * rates[o] for o, k in MIX.items()) / n   # per instruction
        mix_line = (f"mix kernel ({n} instructions per step: {MIX}): measured {rates['mix']:.3f} cycles per "
                    f"instruction, sum of calibrated costs {pred:.3f} -> ratio {rates['mix'] / pred:.3f}")
    # kernel-mix replays (scripts/calib/gen_kmix.py): the additive model on a trace kernel's own mix
    kmix = {}
    kmeta = os.path.join(REPO, "scripts", "calib", "kmix_seq.json")
    for op, meta in (json.load(open(kmeta)).items() if os.path.exists(kmeta) else []):
        if rates.get(op) and all(rates.get(o) for o in meta["ops"]):
            w = {o: k * (2 if o == "cndmask_vcc" else 1) for o, k in meta["ops"].items()}   # instructions
            n = sum(w.values())
            pred = sum(k * rates[o] for o, k in w.items()) / n
            kmix[op] = dict(meta, measured=rates[op], predicted=pred, ratio=rates[op] / pred)
            lines += ["", f"{op} (replay of `{meta['pmc_entry']}`'s VALU mix, {n} ops: {meta['ops']}): measured "
                          f"{rates[op]:.3f} cycles per instruction, sum of calibrated costs {pred:.3f} -> ratio "
                          f"{rates[op] / pred:.3f}"]
    proxies = dict(CLASS_PROXY, other=unclassed)
    cyc = {cls: statistics.mean(rates[o] for o in ps) for cls, ps in proxies.items()}
    other_range = [min(rates[o] for o in unclassed), max(rates[o] for o in unclassed)]
    lines += ["", "Cycles per wave-instruction used by the roofline (class <- calibration kernel(s)):", ""]
    lines += [f"- {cls}: {cyc[cls]:.3f} <- {', '.join(proxies[cls])}" for cls in proxies]
    lines += [f"- other: range {other_range[0]:.3f} .. {other_range[1]:.3f} (bounds of the roofline fraction)"]
    if mix_line:
        lines += ["", mix_line]
    doc = load()
    doc["calibration"] = {"tag": tag, "cycles_per_inst": cyc, "other_range": other_range,
                          "class_counters": CLASS_COUNTERS, "proxies": proxies,
                          "raw": {o: rates.get(o) for o in CALIB_OPS}, "hits": hit_map, "mix": mix_line,
                          "kmix": kmix}
    json.dump(doc, open(OUT_JSON, "w"), indent=1)
    open(os.path.join(REPO, "profiles", f"{tag}_valu_calib.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


def bench(d, tag, workload, note=""):
    import __graft_entry__ as ge

    def sel(name):
        m = re.search(r"(trace_pool|trace_chunks)<rtk::Cfg<(\d+)u, (\w+), (\w+), (\w+), (\w+)(?:, (\w+))?>", name)
        if not m or m.group(6) == "true":      # skip the count_work variant
            return None
        return m.group(1)

    counters, durs, knames = read_counters(d, sel)
    if len(counters) != 1:
        raise SystemExit(f"expected one timed trace kernel, got {list(counters)}")
    (kern, c), = counters.items()
    dur_ns = durs[kern]
    avg_ns = None
    stats = os.path.join(d, "kt", "kt_kernel_stats.csv")
    if os.path.exists(stats):
        shutil.copy(stats, os.path.join(REPO, "profiles", f"{tag}_kernel_stats.csv"))
        for r in csv.DictReader(open(stats)):
            if sel(r["Name"]) == kern:
                avg_ns = float(r["AverageNs"])
    cycles = c["GRBM_GUI_ACTIVE"] / 8.0
    clk = cycles / (dur_ns * 1e-9) / 1e9
    fetch = c.get("FETCH_SIZE", 0.0) * 1024
    write = c.get("WRITE_SIZE", 0.0) * 1024
    dram = 2 * fetch + write
    doc = load()
    src_hash = ge.source_hash()
    kt_log = os.path.join(d, "kt.log")   # the profiled bench's own line names the build it ran
    if os.path.exists(kt_log):
        for line in open(kt_log):
            if line.startswith("{"):
                src_hash = json.loads(line)["roofline"].get("src_hash", src_hash)
    entry = {"tag": tag, "src_hash": src_hash, "workload": workload, "kernel": knames[kern],
             "kernel_ms": (avg_ns or dur_ns) / 1e6, "pmc_dispatch_ms": dur_ns / 1e6, "clock_ghz": clk,
             "dram_bytes": dram, "fetch_bytes_raw": fetch, "write_bytes": write, "counters": c, "note": note}
    doc["entries"] = [e for e in doc["entries"] if not (e["src_hash"] == entry["src_hash"] and
                                                        e["workload"] == workload)] + [entry]
    json.dump(doc, open(OUT_JSON, "w"), indent=1)
    lines = [f"# PMC summary `{tag}` — {knames[kern].split('(')[0]}", "",
             f"workload [scene, W, H, spp, depth, n_gpus, schedule] = {workload}; source hash {entry['src_hash']}",
             f"{note}", "",
             f"kernel-trace average {entry['kernel_ms']:.3f} ms; PMC-pass dispatch {dur_ns / 1e6:.3f} ms; "
             f"clock held GRBM_GUI_ACTIVE/8/t = {clk:.3f} GHz", "",
             "| counter | per launch |", "|---|---|"]
    lines += [f"| {k} | {c[k]:.6g} |" for k in sorted(c)]
    lines += ["", f"DRAM bytes per launch = 2 x FETCH_SIZE + WRITE_SIZE = {dram / 1e6:.2f} MB "
                  f"({dram / (dur_ns * 1e-9) / 1e9:.2f} GB/s = {dram / (dur_ns * 1e-9) / 8e12:.5f} of 8 TB/s)"]
    if "SQ_THREAD_CYCLES_VALU" in c:
        lines.append(f"VALU lane utilisation = SQ_THREAD_CYCLES_VALU / (64 SQ_INSTS_VALU) = "
                     f"{c['SQ_THREAD_CYCLES_VALU'] / (64 * c['SQ_INSTS_VALU']):.3f}")
    cal = doc.get("calibration")
    if cal:
        import bench as bn
        need = bn.valu_issue_cycles(c, cal)
        lines.append(f"VALU issue cycles the mix needs (calibration `{cal['tag']}` class means) = {need:.4g} SIMD-cycles; "
                     f"launch = {N_SIMDS} x {cycles:.4g} = {N_SIMDS * cycles:.4g} -> VALU issue roofline "
                     f"fraction {need / (N_SIMDS * cycles):.3f}")
        m = re.search(r"Cfg<(\d+)u, (\w+), (\w+), (\w+), (\w+), (\w+)>, (true|false)(?:, (true|false))?>", knames[kern])
        isa = (bn.isa_prices(entry["src_hash"], int(m.group(1)), 2 if m.group(7) == "true" else 1,
                             int(m.group(2) == "true"), int(m.group(4) == "true"), ring=m.group(8) == "true")
               if m else None)
        if isa:
            fr = [bn.valu_issue_cycles(c, cal, isa=isa, bound=b) / (N_SIMDS * cycles) for b in (0, -1, 1)]
            lines.append(f"priced from the kernel's own instruction mix (profiles/isa_mix.json): fraction {fr[0]:.3f} "
                         f"(classes at their low / high static-mix prices: {fr[1]:.3f} .. {fr[2]:.3f}); the additive "
                         f"model's check on a saturated mixed stream: {cal.get('mix')}")
        rp = bn.replay_price(cal, int(m.group(1))) if m else None
        if rp:
            lines.append(f"priced at the measured rate of this kernel's mix replayed at saturation "
                         f"({bn.KMIX_OF[int(m.group(1))]}: {rp:.3f} cycles per instruction): fraction "
                         f"{c['SQ_INSTS_VALU'] * rp / (N_SIMDS * cycles):.3f}")
        lines.append(f"(naive 4 x SQ_ACTIVE_INST_VALU / SIMD-cycles = "
                     f"{4 * c.get('SQ_ACTIVE_INST_VALU', 0) / (N_SIMDS * cycles):.3f})")
    open(os.path.join(REPO, "profiles", f"{tag}_pmc.md"), "w").write("\n".join(lines) + "\n")
    print("\n".join(lines))


if __name__ == "__main__":
    mode = sys.argv[1]
    if mode == "calib":
        calib(os.path.join(REPO, "gpurun_out", sys.argv[2]), sys.argv[3])
    else:
        bench(os.path.join(REPO, "gpurun_out", sys.argv[2]), sys.argv[3], [int(x) for x in sys.argv[4].split(",")],
              sys.argv[5] if len(sys.argv) > 5 else "")
