"""The multi-GPU partition on CPU: world_size-2 `gloo` processes each render
their interleaved tiles (rt_shard_pixels, the partition
rt_render_shard_device uses) into a COMPACT accumulator of their own pixels,
and rtamd.dist.gather_frame — the exchange bench.py runs over RCCL — gathers
them onto rank 0 and scatters them into the frame, which must equal the
single-process frame bit for bit.  There is no GPU here, so each rank's
compact accumulator comes from the oracle; the GPU side of the same
partition is test_gpu_parity.py::test_shards_union_bitwise and
::test_compact_shards_match_frame."""
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


def _worker(rank, world, port, out_path, nx, ny):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "scheme-raytrace_amd"))
    sys.path.insert(0, os.path.join(root, "oracle"))
    import torch
    import torch.distributed as dist

    import oracle
    from rtamd import dist as rdist
    from rtamd import scenes

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    scene = scenes.random_scene(nx, ny)
    o = oracle.build_scene(scene)
    pix = rdist.shard_pixels(nx, ny, world)[rank]
    full = np.zeros(nx * ny * 3)
    o.render_pixels(nx, ny, 0, SPP, SEED, full, pix.astype(np.uint32))
    local = torch.from_numpy(np.ascontiguousarray(full.reshape(-1, 3)[pix].ravel()))
    assert local.numel() == rdist.local_size(nx, ny, rank, world)
    frame = rdist.gather_frame(local, nx, ny, rank, world)
    if rank == 0:
        np.save(out_path, frame.numpy())
    else:
        assert frame is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,nx,ny", [(2, NX, NY), (3, 37, 21)])
def test_gloo_tile_shards_reassemble_bitwise(world, nx, ny, tmp_path, oracle_mod):
    """Ragged frames (37x21: partial edge tiles, unequal shard sizes) included."""
    from rtamd import scenes
    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(world, _free_port(), out, nx, ny), nprocs=world, join=True)
    got = np.load(out)
    ref, _ = oracle_mod.build_scene(scenes.random_scene(nx, ny)).render(nx, ny, 0, SPP, SEED)
    assert np.array_equal(got, ref)


def test_shard_pixels_partition_the_frame():
    """Every pixel belongs to exactly one shard, for ragged sizes and several world sizes."""
    from rtamd import dist as rdist
    for nx, ny in [(40, 24), (37, 21), (1920, 1080), (5, 3)]:
        for world in (1, 2, 3, 8):
            pix = np.concatenate(rdist.shard_pixels(nx, ny, world))
            assert np.array_equal(np.sort(pix), np.arange(nx * ny))
