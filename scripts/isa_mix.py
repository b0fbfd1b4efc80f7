#!/usr/bin/env python3
"""Price the trace kernel's "other" VALU instructions (those no SQ_INSTS_VALU_* class counter
counts: moves, selects, compares, bit ops, min/max, ...) from its own instruction mix.

The roofline (bench.py) needs the issue cycles of the launch's VALU mix. The
PMC class counters give exact dynamic counts per class; the rest ("other", ~45 % of VALU
instructions on C2) was priced at the mean of a few calibration kernels with bounds 2.35..4.41
cycles. Here the price comes from the kernel's ISA instead:

  1. compile the variant the workload runs (hipcc -S, the library's flags) and take the trace
     kernel's body, block by block, with each block's loop depth (the compiler's annotations);
  2. map every VALU mnemonic to the calibration kernel measuring it (scripts/calib) and, from the
     calibration's PMC pass, to the class counter it increments (none = "other");
  3. price "other" as the mean issue cost of its static instructions, weighted two ways — every
     instruction of the bounce loop once (loop depth >= 1), and only the inner loops' (depth >= 2:
     node visits, leaf tests, rejection loops, where the dynamic count concentrates) — which
     bound the price; their mean is the point estimate.

usage: python scripts/isa_mix.py [--variant spheres|final|rectinst|media|all] [--items]
Writes profiles/isa_mix.json {src_hash: {variant/kernel: {...}}} (bench.py reads it).
"""
import argparse
import collections
import json
import os
import re
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
OUT = os.path.join(REPO, "profiles", "isa_mix.json")
PMC_JSON = os.path.join(REPO, "profiles", "pmc.json")
FEAT = {"spheres": 0, "rectinst": 35, "media": 103, "final": 287, "all": 4095}

# mnemonic (regex on the opcode, without the _e32/_e64 suffix) -> calibration op
OPMAP = [
    (r"v_mov_b32|v_readfirstlane_b32|v_readlane_b32|v_writelane_b32|v_mov_b32_dpp", "mov_b32"),
    (r"v_mov_b64", "mov_b64"),
    (r"v_xor_b32|v_not_b32|v_xad_u32", "b32_xor"),
    (r"v_and_b32|v_and_or_b32", "and_b32"),
    (r"v_or_b32|v_or3_b32|v_lshl_or_b32", "or_b32"),
    (r"v_bitop3_b32|v_bitop3_b16|v_perm_b32", "bitop3_b32"),
    (r"v_lshlrev_b32|v_lshl_add_u32", "lshl_b32"),
    (r"v_lshrrev_b32|v_ashrrev_i32", "lshr_b32"),
    (r"v_alignbit_b32|v_alignbyte_b32", "alignbit_b32"),
    (r"v_cndmask_b32_e32", "cndmask_e32"),
    (r"v_cndmask_b32_e64|v_cndmask_b32", "cndmask"),
    (r"v_cmp_class_f64|v_cmp_class_f32", "cmp_class_f64"),
    (r"v_cmpx?_\w+_f64", "cmp_f64"),
    (r"v_cmpx?_\w+_f32", "cmp_f32"),
    (r"v_cmpx?_\w+_[iu](32|64|16)", "cmp_i32"),
    (r"v_max_f64|v_min_f64", "max_f64"),
    (r"v_max3_f32|v_min3_f32|v_maximum3_f32|v_minimum3_f32", "max3_f32"),
    (r"v_med3_f32|v_med3_[iu]32", "med3_f32"),
    (r"v_max_f32|v_min_f32|v_max_[iu]32|v_min_[iu]32", "min_f32"),
    (r"v_lshlrev_b64", "lshl_b64"),
    (r"v_lshrrev_b64|v_ashrrev_i64", "lshr_b64"),
    (r"v_lshl_add_u64", "lshl_add_u64"),
    (r"v_mad_u64_u32|v_mad_i64_i32", "mad_u64_u32"),
    (r"v_ldexp_f64|v_frexp_\w+_f64|v_fract_f64|v_floor_f64|v_rndne_f64|v_trunc_f64|v_ceil_f64", "ldexp_f64"),
    (r"v_div_scale_f64", "div_scale_f64"),
    (r"v_div_fmas_f64", "div_fmas_f64"),
    (r"v_div_fixup_f64", "div_fixup_f64"),
    (r"v_mbcnt_\w+", "mbcnt_lo"),
    (r"v_mul_hi_u32|v_mul_hi_i32", "mul_hi_u32"),
    (r"v_mul_lo_u32|v_mul_u32_u24|v_mul_i32_i24", "i32_mul"),
    (r"v_cvt_f32_f64", "cvt_f32_f64"),
    (r"v_cvt_\w+", "cvt_f64_u32"),
    (r"v_sub_u32|v_subrev_u32|v_sub_co_u32|v_subrev_co_u32|v_subb_co_u32|v_sub_i32", "sub_u32"),
    (r"v_add_u32|v_add_co_u32|v_addc_co_u32|v_add3_u32|v_add_i32|v_add_lshl_u32", "i32_add"),
    (r"v_bfe_u32|v_bfe_i32|v_bfi_b32", "bfe_u32"),
    (r"v_fmac_f64", "fmac_f64"),
    (r"v_fma_f64", "f64_fma"),
    (r"v_add_f64", "f64_add"),
    (r"v_mul_f64", "f64_mul"),
    (r"v_rsq_f64", "rsq_f64"),
    (r"v_rcp_f64", "f64_rcp"),
    (r"v_sqrt_f64", "f64_sqrt"),
    (r"v_pk_fma_f32|v_pk_mul_f32|v_pk_add_f32", "pk_fma_f32"),
    (r"v_fma_f32|v_fmac_f32|v_fmamk_f32|v_fmaak_f32", "f32_fma"),
    (r"v_mul_f32", "mul_f32"),
    (r"v_add_f32|v_sub_f32|v_subrev_f32", "f32_add"),
    (r"v_(rcp|rsq|sqrt|exp|log|sin|cos)(_iflag)?_f32", "f32_rcp"),
]


def calib_op(mnemonic):
    m = re.sub(r"_(e32|e64|sdwa|dpp)$", "", mnemonic) if not mnemonic.startswith("v_cndmask") else mnemonic
    for pat, op in OPMAP:
        if re.fullmatch(pat, m):
            return op
    return None


def kernel_asm(variant, items, slab32=1, nall=1, ring=False):
    import __graft_entry__ as ge
    src = os.path.join(ge.CSRC, f"trace_v_{variant}.hip")
    out = f"/tmp/isa_mix_{variant}.s"
    flags = [f for f in ge.CXXFLAGS if f not in ("-Wall", "-Wno-unused-function")]
    subprocess.run(["/opt/rocm/bin/hipcc", *flags, "--cuda-device-only", "-S", src, "-o", out], check=True,
                   capture_output=True)
    lines = open(out).read().splitlines()
    f = FEAT[variant]
    name = re.compile(r"^(_ZN3rtk10trace_poolINS_3CfgILj%dELb%dELb1ELb%dELb0ELb0EEELb%dELb%dEEE\S*):"
                      % (f, slab32, nall, int(items), int(ring)))
    start = next(i for i, l in enumerate(lines) if name.match(l))
    end = next(i for i in range(start + 1, len(lines)) if lines[i].strip().startswith(".size"))
    return name.match(lines[start]).group(1), lines[start:end]


def mix(lines):
    """{depth: Counter(mnemonic)} over the kernel's VALU instructions (block loop depth from the
    compiler's '; in Loop: ... Depth=N' / 'Loop Header: Depth=N' annotations)."""
    by_depth = collections.defaultdict(collections.Counter)
    depth = 0
    for l in lines:
        if re.match(r"^(\.LBB\S+:|; %bb\.\d+:)", l):
            m = re.search(r"Depth=(\d+)", l)
            depth = int(m.group(1)) if m else 0
            continue
        m = re.match(r"^\s+(v_[a-z0-9_]+)", l)
        if m:
            by_depth[depth][m.group(1)] += 1
    return by_depth


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--variant", default="spheres", choices=sorted(FEAT))
    ap.add_argument("--items", action="store_true", help="the item-pool kernel (default: the per-sample pool)")
    ap.add_argument("--ring", action="store_true", help="the per-sample pool reducing in the kernel (RT_OPT_POOL_RING)")
    ap.add_argument("--slab32", type=int, default=1, help="0: the f64-slab instantiation (scenes without BVH nodes)")
    ap.add_argument("--nall", type=int, default=1, help="0: the partial-TLAS instantiation (no TLAS in LDS)")
    a = ap.parse_args()
    import __graft_entry__ as ge
    cal = json.load(open(PMC_JSON))["calibration"]
    raw, hits = cal["raw"], cal.get("hits", {})
    kname, lines = kernel_asm(a.variant, a.items, a.slab32, a.nall, a.ring)
    by_depth = mix(lines)
    unknown = collections.Counter()

    cost = dict(raw)
    # a v_cndmask_b32_e32 reads the vcc a v_cmp just wrote: the calibrated pair (cndmask_vcc,
    # 2 instructions) less the compare
    if cost.get("cndmask_vcc") and cost.get("cmp_f32"):
        cost["cndmask_e32"] = max(2 * cost["cndmask_vcc"] - cost["cmp_f32"], 0.0)
    counter_of = {op: (h[0] if h else None) for op, h in hits.items()}
    counter_of["cndmask_e32"] = None

    def price(min_depth):
        """{class counter or 'other': (mean cost, static count, {op: count})} over blocks at
        loop depth >= min_depth"""
        acc = collections.defaultdict(lambda: [0.0, 0.0, collections.Counter()])
        for d, cnt in by_depth.items():
            if d < min_depth:
                continue
            for mn, k in cnt.items():
                op = calib_op(mn)
                if op is None or cost.get(op) is None or op not in counter_of:
                    unknown[mn] += k
                    continue
                cls = counter_of[op] or "other"
                a = acc[cls]
                a[0] += k * cost[op]
                a[1] += k
                a[2][op] += k
        return {c: (a[0] / a[1], a[1], dict(a[2].most_common())) for c, a in acc.items() if a[1]}

    d1, d2 = price(1), price(2)
    classes = sorted(set(d1) | set(d2))
    est = {"kernel": kname, "calibration": cal["tag"], "classes": {}, "unpriced_mnemonics": dict(unknown.most_common(20))}
    for c in classes:
        p1 = d1.get(c, (None, 0, {}))[0]
        p2 = d2.get(c, (None, 0, {}))[0]
        ps = [p for p in (p1, p2) if p is not None]
        est["classes"][c] = {"price": sum(ps) / len(ps), "range": [min(ps), max(ps)], "depth1": d1.get(c), "depth2": d2.get(c)}
    o = est["classes"]["other"]
    est.update({"other_price": o["price"], "other_range": o["range"]})
    p1, p2 = (o["depth1"] or (None,))[0], (o["depth2"] or (None,))[0]
    n1, n2 = (o["depth1"] or (0, 0))[1], (o["depth2"] or (0, 0))[1]
    doc = json.load(open(OUT)) if os.path.exists(OUT) else {}
    h = ge.source_hash()
    doc.setdefault(h, {})[f"{a.variant}/{'items' if a.items else 'ring' if a.ring else 'pool'}/s{a.slab32}n{a.nall}"] = est
    json.dump(doc, open(OUT, "w"), indent=1)
    print(f"{kname}: other priced {p1:.3f} (bounce loop, {int(n1)} static instructions) .. {p2:.3f} "
          f"(inner loops, {int(n2)}); estimate {est['other_price']:.3f}")
    for c, v in est["classes"].items():
        print(f"  {c:24s} {v['price']:.3f}  range {v['range'][0]:.3f} .. {v['range'][1]:.3f}")
    if unknown:
        print("unpriced:", dict(unknown.most_common(12)))


if __name__ == "__main__":
    main()
