"""The N > 1 path through the HIP library: two rank processes, both on
device 0, each render their interleaved row shard through librtiow_amd.so and rank 0
gathers the shards over gloo and re-interleaves them. The frame must equal the
one-process render bit for bit (every draw is keyed by pixel and sample).

This file sorts first among the GPU tests so the rank processes start before this test
process has touched the GPU (they are children started with subprocess, never an exec
of this process)."""
import os
import socket
import subprocess
import sys

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run_ranks(world, scene, W, H, spp, out, block=1):
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_free_port()), WORLD_SIZE=str(world))
    procs = [subprocess.Popen([sys.executable, "-m", "tests.multirank_worker", str(scene), str(W), str(H), str(spp),
                               out, str(block)], cwd=REPO, env=dict(env, RANK=str(r)))
             for r in range(world)]
    rcs = []
    for p in procs:
        try:
            rcs.append(p.wait(timeout=400))   # a fresh box's first `import torch` takes minutes
        except subprocess.TimeoutExpired:
            p.kill()
            rcs.append(-9)
    return rcs


@pytest.mark.timeout(900)
def test_hip_row_shards_over_processes_equal_single_render(rt, tmp_path):
    scene, W, H, spp = 7, 96, 53, 8
    frames = {}
    # single-row interleave (world 2) and bench.py's 8-row bands (world 3; 53 rows: a cut last band)
    for world, block in ((2, 1), (3, 8)):   # every rank process runs before this process touches the GPU
        out = str(tmp_path / f"frame{world}.npy")
        rcs = _run_ranks(world, scene, W, H, spp, out, block)
        assert rcs == [0] * world, (world, rcs)
        frames[world] = np.load(out)
    img, _ = rt.render_scene(scene, W, H, spp, 50, out_format=rt.RT_OUT_F64)
    for world, frame in frames.items():
        assert np.array_equal(frame, img), world
