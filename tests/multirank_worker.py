"""One rank of tests/test_gpu_0_multirank.py, run as its own process (python -m
tests.multirank_worker): renders its interleaved row shard through librtiow_amd.so on
device 0 (the C ABI, render_device into a torch tensor on a torch stream, as bench.py's
step does), and rank 0 gathers the host copies of every shard over gloo, re-interleaves
them (rtiow_amd.assemble_rows) and saves the frame."""
import os
import sys

import numpy as np
import torch
import torch.distributed as dist

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)


def main():
    scene, W, H, spp, out = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), sys.argv[5]
    block = int(sys.argv[6]) if len(sys.argv) > 6 else 1   # row_block: bands of rows, as bench.py shards
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import __graft_entry__ as ge
    rt = ge.import_binding()
    r = rt.Renderer(0)
    w = rt.World(1).build_scene(scene)
    cam, bg = rt.scene_camera(scene, W, H)
    r.upload(w)
    rows = rt.rows_in_shard(H, rank, world, block)
    rows_max = max(rt.rows_in_shard(H, q, world, block) for q in range(world))
    slab = torch.zeros((rows_max, W, 3), dtype=torch.float64, device="cuda:0")
    stream = torch.cuda.Stream(torch.device("cuda", 0))
    p = rt.Renderer.params(W, H, spp, 50, bg, 1, row_begin=rank, row_stride=world, out_format=rt.RT_OUT_F64,
                           row_block=block)
    with torch.cuda.stream(stream):
        r.render_device(cam, p, slab.data_ptr(), stream.cuda_stream)
    torch.cuda.synchronize()
    host = slab.cpu()
    assert rows <= rows_max
    gathered = [torch.empty_like(host) for _ in range(world)] if rank == 0 else None
    dist.gather(host, gathered, dst=0)
    if rank == 0:
        frame = rt.assemble_rows([g.numpy() for g in gathered], H, world, row_block=block)
        np.save(out, frame)
    dist.barrier()
    dist.destroy_process_group()
    r.close()


if __name__ == "__main__":
    main()
