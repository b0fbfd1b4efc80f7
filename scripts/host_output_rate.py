#!/usr/bin/env python3
"""C2 through the host-buffer boundary (rt_render, out_on_device = 0: the frame comes back
over PCIe into caller memory): wall time per call vs the trace kernel's HIP-event time."""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
import numpy as np  # noqa: E402
import __graft_entry__ as ge  # noqa: E402

rt = ge.import_binding()
W, H, spp = 1200, 800, 500
world = rt.World(1).build_scene(0)
cam, bg = rt.scene_camera(0, W, H)
r = rt.Renderer(0)
r.upload(world)
p = rt.Renderer.params(W, H, spp, 50, bg, 1, out_format=rt.RT_OUT_F32)
out = np.empty((H, W, 3), np.float32)
r.render(cam, p, out)
walls, kernels = [], []
for _ in range(3):
    t0 = time.perf_counter()
    r.render(cam, p, out)
    walls.append((time.perf_counter() - t0) * 1e3)
    kernels.append(r.stats().kernel_ms)
w, k = float(np.median(walls)), float(np.median(kernels))
print(f"host-output rt_render C2: wall {w:.2f} ms/frame ({W * H * spp / w / 1e3:.1f} Msamples/s), "
      f"trace kernel {k:.2f} ms; frame {W * H * 12 / 1e6:.1f} MB f32")
