"""The N > 1 path through the HIP library: two rank processes, both on
device 0, each render their interleaved row shard through librtiow_amd.so and rank 0
gathers the shards over gloo and re-interleaves them. The frame must equal the
one-process render bit for bit (every draw is keyed by pixel and sample).

bench.py's own N > 1 branch runs here too: `torch.distributed.run
--nproc-per-node 2 bench.py --gpus 2 --transport gloo --device 0` (both ranks on the one
GPU of the box; gloo, since RCCL refuses two ranks on one device) — its shard, gather,
re-interleave, barrier and max-over-ranks timing — against bench.py at N = 1, whose default
path is the library's rt_render_gather over a world-1 RCCL communicator.

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


def _bench(tmp_path, world, tag, extra=(), rccl=False):
    """bench.py as child processes (N > 1: torch.distributed.run, one child per rank), a
    small random-scene workload; returns (JSON line of rank 0, frame, PPM bytes). rccl: one
    rank under torch.distributed.run with --force-dist and the default transport (the library's
    RCCL communicator, the unique id broadcast over torch's gloo control plane)."""
    frame, ppm = str(tmp_path / f"{tag}.npy"), str(tmp_path / f"{tag}.ppm")
    args = ["bench.py", "--gpus", str(world), "--device", "0", "--scene", "0", "--width", "160", "--height", "90",
            "--spp", "8", "--depth", "50", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-count",
            "--frame-npy", frame, "--ppm", ppm, *extra]
    if rccl:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node=1",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), *args, "--force-dist"]
    elif world > 1:
        cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
               "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), *args, "--transport", "gloo"]
    else:
        cmd = [sys.executable, *args]
    env = {k: v for k, v in os.environ.items() if k not in ("RANK", "WORLD_SIZE", "LOCAL_RANK", "MASTER_ADDR",
                                                               "MASTER_PORT")}
    p = subprocess.run(cmd, cwd=REPO, env=env, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, (world, p.returncode, p.stderr[-3000:])
    import json
    lines = [l for l in p.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]   # rank 0 alone prints the JSON line
    return json.loads(lines[0]), np.load(frame), open(ppm, "rb").read()


@pytest.mark.timeout(1300)
def test_bench_py_n2_branch_equals_n1(tmp_path):
    """bench.py --gpus 2 (two ranks on device 0, gloo gather of the 8x8 tile shards, 90 rows:
    a cut last tile row) and --gpus 3 --shard rows (interleaved rows) write the N = 1 frame bit
    for bit, and their JSON lines report n_gpus (runs before this test process touches the
    GPU: every GPU user here is a child process)."""
    j2, f2, p2 = _bench(tmp_path, 2, "n2")
    j3, f3, p3 = _bench(tmp_path, 3, "n3", extra=("--shard", "rows"))
    j1, f1, p1 = _bench(tmp_path, 1, "n1")
    assert j2["n_gpus"] == 2 and j3["n_gpus"] == 3 and j1["n_gpus"] == 1
    assert j2["steps"] == 2 and j2["value"] > 0 and j2["ms_per_step"] > 0
    assert "gloo" in j2["config"]["parallelism"] and "8x8 tiles (cost order)" in j2["config"]["parallelism"]
    assert "rows" in j3["config"]["parallelism"]
    assert f2.shape == f3.shape == f1.shape == (90, 160, 3)
    assert np.array_equal(f2, f1) and np.array_equal(f3, f1)
    assert p2 == p1 and p3 == p1
    # the N > 1 line carries the value with the cost pass amortised (the
    # headline, consistent with ms_per_step) and without it
    pass_s = j2["detail"]["tile_order_pass_s"]
    assert pass_s > 0 and j2["value_steady"] > j2["value"] and "amortised" in j2["value_basis"]
    samples = 160 * 90 * 8 * 2
    assert abs(j2["value"] - samples / (j2["ms_per_step"] * 2e-3) / 1e6) <= 1e-3 * j2["value"] + 1e-3
    assert abs(samples / (j2["value_steady"] * 1e6) + pass_s - samples / (j2["value"] * 1e6)) < 1e-3
    # N = 1: no cost pass, one value; its path is rt_render_gather over a world-1 communicator,
    # which renders straight into the frame (RT_OPT_COMM_DIRECT)
    assert j1["value"] == j1["value_steady"] and j1["detail"]["tile_order_pass_s"] is None
    assert "rt_render_gather of a world of one" in j1["config"]["parallelism"]


@pytest.mark.timeout(900)
def test_bench_py_cost_order_survives_chunks_and_f32(tmp_path):
    """the cost pass needs f64 and a pool schedule (the chunk schedule counts no tile
    costs; count_work in f32 is refused on the Cornell variant). Under --schedule chunks and
    --precision f32 on the Cornell box, two gloo ranks still agree on a cost order (the pass runs f64
    / POOL and restores the settings), and the frame equals N = 1's bit for bit."""
    extra = ("--scene", "5", "--schedule", "chunks", "--precision", "f32")
    j2, f2, _ = _bench(tmp_path, 2, "c3n2", extra=extra)
    j1, f1, _ = _bench(tmp_path, 1, "c3n1", extra=extra)
    assert j2["config"]["tile_order"] == "cost" and j2["detail"]["schedule"] == 0
    assert j2["dtype"] == "f32" and np.array_equal(f2, f1)


@pytest.mark.timeout(900)
def test_bench_py_rccl_branch_at_world_size_1(tmp_path):
    """bench.py's distributed branch with the product's transport,
    the library's RCCL communicator, executed at world size 1 on the box's one GPU: torch's gloo
    control plane broadcasts the RCCL unique id, rt_comm_init_rank, rt_comm_tile_order (the count
    pass of the rank's shard, the RCCL all-reduce of the tile costs, the cost order set),
    rt_render_gather per step (the shard, the RCCL gather, the reorder kernel), the barriers and the
    MAX all-reduce. Its frame and PPM equal the plain N = 1 run (rt_render_gather of a world of one:
    straight into the frame), the same with --comm-direct 0 (the raster tile shard, the RCCL
    gather, the reorder kernel) and the --transport none run (rt_render) bit for bit."""
    jd, fd, pd = _bench(tmp_path, 1, "rccl1", extra=("--tile-order", "cost"), rccl=True)
    j1, f1, p1 = _bench(tmp_path, 1, "plain1")
    js, fs, ps = _bench(tmp_path, 1, "shard1", extra=("--comm-direct", "0"))
    jn, fn, pn = _bench(tmp_path, 1, "none1", extra=("--transport", "none"))
    assert jd["n_gpus"] == 1 and "RCCL gather (library communicator" in jd["config"]["parallelism"]
    assert "8x8 tiles (cost order)" in jd["config"]["parallelism"] and jd["config"]["tile_order"] == "cost"
    assert jd["detail"]["tile_order_pass_s"] > 0
    assert jd["distributed"] == {"transport": "RCCL (library communicator)", "control_plane": "torch.distributed gloo",
                                 "world_size": 1, "forced_at_world_1": True}
    pr = jd["per_rank"]
    assert len(pr) == 1 and pr[0]["kernel_ms"] > 0 and pr[0]["gather_ms"] >= 0 and pr[0]["samples"] >= 160 * 90 * 8
    assert pr[0]["render_ms"] >= pr[0]["kernel_ms"]
    assert "per_rank" not in j1 and "rt_render_gather of a world of one" in j1["config"]["parallelism"]
    assert j1["detail"]["gather_ms_mean"] <= js["detail"]["gather_ms_mean"]
    assert "8x8 tiles (raster order)" in js["config"]["parallelism"] and "RCCL gather" in js["config"]["parallelism"]
    assert "no gather" in jn["config"]["parallelism"] and jn["detail"]["gather_ms_mean"] is None
    assert fd.dtype == np.float64 and fd.shape == f1.shape == fs.shape == fn.shape == (90, 160, 3)
    assert np.array_equal(fd, f1) and np.array_equal(fs, f1) and np.array_equal(fn, f1)
    assert pd == p1 == ps == pn


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
