"""The multi-GPU partition on CPU: world_size-2 `gloo` processes each render
their interleaved tiles (rt_shard_pixels, the partition rt_render_device's
shard arguments use) into a full-frame f64 accumulator and reduce to rank 0,
as bench.py does over RCCL; the gathered frame equals the single-process
frame bit for bit.  The compute here is the oracle (there is no GPU in this
test); the GPU path of the same partition is covered by
test_gpu_parity.py::test_shards_union_bitwise."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

NX, NY, SPP, SEED = 40, 24, 2, 0x5EED0002


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_path):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "scheme-raytrace_amd"))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch
    import torch.distributed as dist

    import oracle
    from rtamd import gpu, scenes

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scene = scenes.random_scene(NX, NY)
    o = oracle.build_scene(scene)
    acc = np.zeros(NX * NY * 3)
    o.render_pixels(NX, NY, 0, SPP, SEED, acc, gpu.shard_pixels(NX, NY, rank, world))
    t = torch.from_numpy(acc)
    dist.reduce(t, dst=0, op=dist.ReduceOp.SUM)
    if rank == 0:
        np.save(out_path, t.numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2])
def test_gloo_tile_shards_reassemble_bitwise(world, tmp_path, oracle_mod):
    from rtamd import scenes
    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    got = np.load(out)
    ref, _ = oracle_mod.build_scene(scenes.random_scene(NX, NY)).render(NX, NY, 0, SPP, SEED)
    assert np.array_equal(got, ref)
