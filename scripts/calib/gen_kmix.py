#!/usr/bin/env python3
"""Replay a trace kernel's VALU instruction mix as a calibration kernel.

The roofline prices the kernel's VALU instructions class by class at the issue cost each
class has alone at saturation (scripts/calib). Whether those costs add up for a *mix* is what
this checks, on the kernel's own mix: the dynamic class shares come from the kernel's PMC
pass (profiles/pmc.json entry), the instructions inside each class from its ISA
(profiles/isa_mix.json, loop depth >= 1), and a sequence of N calibration ops with those
shares (largest remainder, spread out by a stride schedule) becomes the KMIX_<name> kernel of
valu_calib.hip. Its measured cycles per instruction against the sum of its ops' calibrated
costs is the additive model's error on that mix.

usage: python scripts/calib/gen_kmix.py   (writes scripts/calib/kmix_seq.h and kmix_seq.json)
"""
import json
import os

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
N = 40
# name -> (PMC entry tag, isa_mix key); RT_KMIX_TAGS="c2=tag,c3=tag,c4=tag" picks other PMC entries
MIXES = {"c2": ("r03j_c2", "spheres/pool/s1n1"), "c4": ("r03j_c4", "final/pool/s1n1")}
if os.environ.get("RT_KMIX_TAGS"):
    KEYS = {"c2": "spheres/pool/s1n1", "c3": "rectinst/pool/s0n0", "c4": "final/pool/s1n1"}
    MIXES = {k: (v, KEYS[k]) for k, v in (x.split("=") for x in os.environ["RT_KMIX_TAGS"].split(","))}
ENUM = {  # calibration op name -> valu_calib.hip enum
    "f64_fma": "F64_FMA", "f64_add": "F64_ADD", "f64_mul": "F64_MUL", "f64_rcp": "F64_RCP", "f64_sqrt": "F64_SQRT",
    "f32_fma": "F32_FMA", "f32_add": "F32_ADD", "f32_rcp": "F32_RCP", "i32_add": "I32_ADD", "i32_mul": "I32_MUL",
    "b32_xor": "B32_XOR", "cndmask": "CNDMASK", "mov_b32": "MOV_B32", "cmp_f64": "CMP_F64", "cmp_f32": "CMP_F32",
    "max_f64": "MAX_F64", "min_f32": "MIN_F32", "lshl_b64": "LSHL_B64", "cvt_f64_u32": "CVT_F64_U32",
    "bfe_u32": "BFE_U32", "pk_fma_f32": "PK_FMA_F32", "max3_f32": "MAX3_F32", "med3_f32": "MED3_F32",
    "and_b32": "AND_B32", "or_b32": "OR_B32", "lshl_b32": "LSHL_B32", "lshr_b32": "LSHR_B32",
    "alignbit_b32": "ALIGNBIT", "bitop3_b32": "BITOP3", "mov_b64": "MOV_B64", "cmp_i32": "CMP_I32",
    "ldexp_f64": "LDEXP_F64", "div_scale_f64": "DIV_SCALE_F64", "div_fmas_f64": "DIV_FMAS_F64",
    "div_fixup_f64": "DIV_FIXUP_F64", "mad_u64_u32": "MAD_U64_U32", "lshl_add_u64": "LSHL_ADD_U64",
    "lshr_b64": "LSHR_B64", "mbcnt_lo": "MBCNT_LO", "mul_hi_u32": "MUL_HI_U32", "cvt_f32_f64": "CVT_F32_F64",
    "cmp_class_f64": "CMP_CLASS_F64", "sub_u32": "SUB_U32", "fmac_f64": "FMAC_F64", "mul_f32": "MUL_F32",
    "rsq_f64": "RSQ_F64", "cndmask_e32": "CNDMASK_E32", "cndmask_vcc": "CNDMASK_VCC"}
INSTS = {"cndmask_vcc": 2}   # instructions per op


def op_shares(entry, isa):
    """{calibration op: share of the kernel's dynamic VALU instructions}"""
    c = entry["counters"]
    tot = c["SQ_INSTS_VALU"]
    shares = {}
    classed = 0.0
    for cls, v in isa["classes"].items():
        if cls == "other":
            continue
        n = c.get("SQ_INSTS_VALU_" + cls, 0.0)
        classed += n
        comp = (v["depth1"] or [None, 0, {}])[2]
        w = sum(comp.values())
        for op, k in comp.items():
            shares[op] = shares.get(op, 0.0) + n / tot * k / w
    comp = isa["classes"]["other"]["depth1"][2]
    w = sum(comp.values())
    for op, k in comp.items():
        shares[op] = shares.get(op, 0.0) + (1.0 - classed / tot) * k / w
    return {op: s for op, s in shares.items() if op in ENUM}


def pair_selects(shares):
    """The kernel's v_cndmask_b32_e32 reads the vcc a v_cmp just wrote (alone, a select of an
    unwritten vcc issues at ~22 cycles): replay each as the calibrated cmp + select pair
    (CNDMASK_VCC, 2 instructions), its compare taken from the kernel's compares."""
    s = dict(shares)
    sel = s.pop("cndmask_e32", 0.0)
    for cmp in ("cmp_i32", "cmp_f64", "cmp_f32"):
        take = min(sel, s.get(cmp, 0.0))
        s[cmp] = s.get(cmp, 0.0) - take
        s["cndmask_vcc"] = s.get("cndmask_vcc", 0.0) + take   # pairs (one per 2 instructions)
        sel -= take
    s["cndmask_vcc"] += sel
    return s


def sequence(shares, n=N):
    shares = pair_selects(shares)
    tot = sum(v * INSTS.get(op, 1) for op, v in shares.items())
    # pairs: count slots in instructions; a CNDMASK_VCC op is 2 of them
    shares = {op: v * INSTS.get(op, 1) for op, v in shares.items()}
    exact = {op: s / tot * n / INSTS.get(op, 1) for op, s in shares.items()}   # in ops
    count = {op: int(x) for op, x in exact.items()}
    for op in sorted(exact, key=lambda o: exact[o] - count[o], reverse=True):
        if sum(count[o] * INSTS.get(o, 1) for o in count) + INSTS.get(op, 1) > n:
            continue
        count[op] += 1
    # stride schedule: op k-th copy at position (k + 0.5) / count, so no op runs in a block
    slots = sorted(((k + 0.5) / m, op) for op, m in count.items() if m for k in range(m))
    return [op for _, op in slots], {op: m for op, m in count.items() if m}


def main():
    pmc = json.load(open(os.path.join(REPO, "profiles", "pmc.json")))
    isa_doc = json.load(open(os.path.join(REPO, "profiles", "isa_mix.json")))
    out, meta = [], {}
    for name, (tag, key) in MIXES.items():
        entry = [e for e in pmc["entries"] if e["tag"] == tag][-1]   # the latest entry of that tag
        isa = isa_doc[entry["src_hash"]][key]
        seq, count = sequence(op_shares(entry, isa))
        meta["kmix_" + name] = {"pmc_entry": tag, "isa_mix": key, "src_hash": entry["src_hash"], "ops": count}
        out.append(f"// {name}: the {tag} launch's dynamic class shares x {key}'s in-class ISA mix, {len(seq)} ops")
        out.append(f"#define KMIX_{name.upper()}_SEQ " + ", ".join(ENUM[o] for o in seq))
        print(name, count)
    open(os.path.join(HERE, "kmix_seq.h"), "w").write(
        "// generated by scripts/calib/gen_kmix.py: do not edit\n" + "\n".join(out) + "\n")
    json.dump(meta, open(os.path.join(HERE, "kmix_seq.json"), "w"), indent=1)


if __name__ == "__main__":
    main()
