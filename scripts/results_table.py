#!/usr/bin/env python3
"""DESIGN.md §7's results table from bench logs (one JSON line each).

usage: python scripts/results_table.py PREFIX [cN=OTHER_PREFIX ...]
       (reads profiles/PREFIX{bench_c1..c5,f32_c2..c4}.log; cN=OTHER takes config N's f64 line from
       profiles/OTHERbench_cN.log instead)
"""
import json
import os
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def line(path):
    try:
        for l in open(path):
            if l.startswith("{"):
                return json.loads(l)
    except OSError:
        return None
    return None


def main():
    pre = sys.argv[1]
    over = dict(a.split("=", 1) for a in sys.argv[2:])
    names = {"C1": "C1 random 1200×800×10, depth 8", "C2": "**C2 random 1200×800×500** (headline)",
             "C3": "C3 Cornell 800×800×1000", "C4": "C4 final 1920×1080×1000", "C5": "C5 random 4096²×4096"}
    print("| config (BASELINE) | Msamples/s | ms/frame (kernel + reduce) | schedule, batches, waves/SIMD | "
          "VALU-issue frac [range] | lane util | useful | DRAM frac | f32 mode | cpu_baseline (oracle, threads) | "
          "ref. split, 10 threads | parity L∞ |")
    print("|---|---|---|---|---|---|---|---|---|---|---|---|")
    for c in ("C1", "C2", "C3", "C4", "C5"):
        d = line(os.path.join(REPO, "profiles", f"{over.get(c.lower(), pre)}bench_{c.lower()}.log"))
        if d is None:
            continue
        f = line(os.path.join(REPO, "profiles", f"{pre}f32_{c.lower()}.log"))
        x, r = d["detail"], d["roofline"]
        sched = {0: "chunks", 1: "pool", 2: "items"}[x["schedule"]]
        frac = "—" if r.get("frac") is None else f"{r['frac']:.3f} [{r['frac_range'][0]:.3f}, {r['frac_range'][1]:.3f}]"
        cpu = d.get("cpu_baseline") or {}
        t10 = cpu.get("ref_split_t10") or {}
        par = d.get("parity") or {}
        print(f"| {names[c]} | {d['value']:,.0f} | {d['ms_per_step']:.2f} ({x['kernel_ms_mean']:.2f} + {x['reduce_ms']:.2f}) | "
              f"{sched}, {x['n_batches']}, {x['waves_per_simd']} | {frac} | {r.get('valu_lane_util', '—')} | "
              f"{r.get('useful_frac', '—')} | {(r.get('hbm') or {}).get('frac', '—')} | "
              f"{'—' if f is None else format(f['value'], ',.0f')} | "
              f"{cpu.get('value', float('nan')):.2f} ({cpu.get('cores', '—')}) | {t10.get('value', float('nan')):.2f} | "
              f"{par.get('linf', float('nan')):.1e} |")


if __name__ == "__main__":
    main()
