#!/usr/bin/env python3
"""A/B whole library builds (e.g. lib/librtiow_amd.so vs lib/librtiow_exp_*.so built with
__graft_entry__.build_library(extra_flags=[...], name=...)) on one render config.

Each build runs in its own child process (RT_LIB_PATH picks the .so); the children run
one after another, `--rounds` times round-robin, so clock drift spreads over all builds.
Prints per-build median kernel ms and whether the f64 test image equals the first build's.

usage: python scripts/ab_builds.py lib/a.so lib/b.so [--scene 0 --width 1200 --height 800 --spp 500]
       (a build given as lib/a.so@opt9=0,opt1=4294967296 runs with those rt_ctx_set_option
       keys and values, @optsched=2 with that rt_ctx_set_schedule, @optprec=1 the f32 mode; any other NAME=V pair is set
       in the child's environment)
       Times are kernel + reduce ms (the frame's trace launches and their reductions).
"""
import argparse
import hashlib
import json
import os
import subprocess
import sys

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))

CHILD = r"""
import json, os, sys, time
sys.path.insert(0, {repo!r})
import numpy as np
import __graft_entry__ as ge
rt = ge.import_binding()
a = json.loads({args!r})
world = rt.World(1).build_scene(a["scene"])
cam, bg = rt.scene_camera(a["scene"], a["width"], a["height"])
r = rt.Renderer(0)
for k, v in a["opts"].items():
    if k == "sched":
        r.set_schedule(int(v))
    elif k == "prec":
        r.set_precision(int(v))
    else:
        r.set_option(int(k), int(v))
r.upload(world)
img = r.render(cam, rt.Renderer.params(a["width"], a["height"], 2, a["depth"], bg, 1, row_stride=8,
                                       out_format=rt.RT_OUT_F64))
p = rt.Renderer.params(a["width"], a["height"], a["spp"], a["depth"], bg, 1, out_format=rt.RT_OUT_F32)
out = np.empty((a["height"], a["width"], 3), np.float32)
r.render(cam, p, out)
ms, red = [], []
for _ in range(a["reps"]):
    r.render(cam, p, out)
    st = r.stats()
    ms.append(st.kernel_ms + st.reduce_ms)
    red.append(st.reduce_ms)
import hashlib
print("RESULT", json.dumps({{"ms": ms, "reduce_ms": red, "trace_buf_bytes": st.trace_buf_bytes, "n_batches": st.n_batches,
                            "ring_bytes": getattr(st, "ring_bytes", 0), "img": hashlib.sha1(img.tobytes()).hexdigest(),
                            "frame": hashlib.sha1(out.tobytes()).hexdigest()}}))
"""


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("libs", nargs="+")
    ap.add_argument("--scene", type=int, default=0)
    ap.add_argument("--width", type=int, default=1200)
    ap.add_argument("--height", type=int, default=800)
    ap.add_argument("--spp", type=int, default=500)
    ap.add_argument("--depth", type=int, default=50)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--rounds", type=int, default=2)
    a = ap.parse_args()
    base_args = dict(scene=a.scene, width=a.width, height=a.height, spp=a.spp, depth=a.depth, reps=a.reps)
    res = {lib: [] for lib in a.libs}
    red = {lib: [] for lib in a.libs}
    imgs = {}
    for _ in range(a.rounds):
        for lib in a.libs:
            path, _, extra = lib.partition("@")   # lib.so@NAME=V,NAME=V: that build under those env vars
            env = dict(os.environ, RT_LIB_PATH=os.path.abspath(os.path.join(REPO, path)))
            kvs = [kv.split("=", 1) for kv in extra.split(",") if kv]
            env.update((k, v) for k, v in kvs if not k.startswith("opt"))
            code = CHILD.format(repo=REPO, args=json.dumps(dict(base_args, opts={k[3:]: v for k, v in kvs if k.startswith("opt")})))
            out = subprocess.run([sys.executable, "-c", code], env=env, capture_output=True, text=True, timeout=600)
            if out.returncode != 0:
                print(f"{lib}: child failed ({out.returncode})\n{out.stderr[-2000:]}")
                sys.exit(out.returncode if out.returncode > 0 else 1)
            line = [x for x in out.stdout.splitlines() if x.startswith("RESULT ")][-1]
            d = json.loads(line[7:])
            res[lib] += d["ms"]
            red[lib] += d.get("reduce_ms", [])
            imgs[lib] = (d["img"], d.get("frame"))
            print(f"  {lib}: {['%.2f' % m for m in d['ms']]}  buf {d['trace_buf_bytes'] / 2**30:.2f} GiB "
                  f"(ring {d['ring_bytes'] / 2**30:.2f}) batches {d['n_batches']}", flush=True)
    base = imgs[a.libs[0]]
    n = a.width * a.height * a.spp
    for lib in a.libs:
        ms = sorted(res[lib])[len(res[lib]) // 2]
        print(f"{lib}: median {ms:.2f} ms  min {min(res[lib]):.2f}  -> {n / ms / 1e3:.1f} Msamples/s  "
              f"image == {a.libs[0]}: {imgs[lib][0] == base[0]}  whole timed frame == {a.libs[0]}: "
              f"{imgs[lib][1] == base[1]}"
              + (f"  reduce median {sorted(red[lib])[len(red[lib]) // 2]:.3f} ms" if red[lib] else ""))


if __name__ == "__main__":
    main()
