"""Multi-GPU frames: one process per GPU, tile-sharded.

trace-all has no cross-pixel dependence (main.scm:471-491) and the counter RNG
keys every sample by (seed, pixel, sample), so a frame splits into disjoint
pixel sets with no exchange until the end.  Rank r renders the interleaved
16x16 tiles (tx, ty) with (tx + k ty) % world == r (k the smallest odd prime not dividing world;
rt_shard_pixels) into a COMPACT accumulator
— its own pixels only, in shard order (rt_render_shard_device) — and rank 0
gathers the shards over the process group (RCCL over xGMI with the "nccl"
backend; gloo on the CPU) and scatters them into the y-up frame.  Each rank
ships 1/world of the frame instead of a full-frame buffer, and the result is
bit-identical to a one-process render (the pixels are disjoint, nothing is
summed).

``gather_frame`` is the exchange step; bench.py calls it after each rank's
rt_render_shard_device (timing the two apart), tests/test_distributed.py calls
it with gloo on CPU tensors.  On GPUs ("nccl" backend) it runs behind the C
ABI: rt_gather_shards over a librtamd communicator (rt_comm_create, its id
made by rank 0 and broadcast over the process group), which sends each
shard's exact pixel count (grouped send / receive, no padding) and places the
pixels into rank 0's frame on the device; the gloo path (CPU rehearsals) is
the same exchange in torch.distributed.
"""
import numpy as np

from . import gpu

_pix_cache = {}
_dev_cache = {}
_comms = {}


def shard_pixels(nx, ny, world):
    """Per-rank pixel lists (image pixel j = y*nx + x), rank r's in its compact order."""
    key = (nx, ny, world)
    if key not in _pix_cache:
        _pix_cache[key] = [gpu.shard_pixels(nx, ny, r, world).astype(np.int64) for r in range(world)]
    return _pix_cache[key]


def _gather_buffers(nx, ny, world, dtype, dev, frame_dev):
    """The exchange's buffers, made once per (frame, world, device) and kept:
    the padded send buffer, rank 0's receive buffer (one tensor, a row per
    rank), and the scatter's two index lists already on rank 0's device: the
    receive rows' valid pixels (padding skipped) and their frame pixels."""
    import torch
    key = (nx, ny, world, dtype, str(dev), str(frame_dev))
    if key not in _dev_cache:
        pix = shard_pixels(nx, ny, world)
        width = max(len(p) for p in pix)        # collectives move equal-size buffers: pad to the largest shard
        src = np.concatenate([r * width + np.arange(len(p), dtype=np.int64) for r, p in enumerate(pix)])
        dst = np.concatenate(pix)
        _dev_cache[key] = {
            "send": torch.zeros(3 * width, dtype=dtype, device=dev),
            "recv": None,                       # rank 0 only (gather_frame)
            "src": torch.from_numpy(src).to(frame_dev), "dst": torch.from_numpy(dst).to(frame_dev),
            "width": width,
        }
    return _dev_cache[key]


def gather_frame(local, nx, ny, rank, world, group=None, out=None):
    """Gather every rank's compact accumulator (a 1-D float64 tensor of
    3 x its pixel count) onto rank 0 and scatter it into an nx*ny*3 frame
    (``out`` if given, else a new tensor on local's device).  Returns the
    frame on rank 0, None on other ranks.  Shards differ by at most one
    16x16 tile, so padding them to equal size moves < 6 KB more per rank;
    rank 0 then places all of them with one gather and one scatter."""
    import torch
    import torch.distributed as dist

    pix = shard_pixels(nx, ny, world)
    counts = [len(p) for p in pix]
    if local.numel() != 3 * counts[rank]:
        raise ValueError("rank %d holds %d values, its shard has %d pixels" % (rank, local.numel(), counts[rank]))
    if dist.get_backend(group) != "gloo":          # GPUs: the C ABI's RCCL gather (rt_gather_shards)
        if rank == 0 and out is None:
            out = torch.empty(nx * ny * 3, dtype=local.dtype, device=local.device)
        if rank == 0 and out.numel() != nx * ny * 3:
            raise ValueError("out must hold nx*ny*3 values")
        comm = communicator(rank, world, group, local.device)
        comm.gather_shards(nx, ny, local.data_ptr(), out.data_ptr() if rank == 0 else 0,
                           torch.cuda.current_stream(local.device).cuda_stream)
        return out if rank == 0 else None
    # gloo (CPU tests, one-GPU rehearsals of the multi-process bench) gathers host copies
    dev = torch.device("cpu")
    B = _gather_buffers(nx, ny, world, local.dtype, dev, local.device)
    send = B["send"]
    send[:local.numel()].copy_(local)
    if rank == 0 and B["recv"] is None:
        B["recv"] = torch.empty(world, send.numel(), dtype=send.dtype, device=dev)
    dist.gather(send, gather_list=list(B["recv"].unbind(0)) if rank == 0 else None, dst=0, group=group)
    if rank != 0:
        return None
    if out is None:
        out = torch.empty(nx * ny * 3, dtype=local.dtype, device=local.device)
    if out.numel() != nx * ny * 3:
        raise ValueError("out must hold nx*ny*3 values")
    recv = B["recv"].to(local.device).view(-1, 3)     # the shards cover every pixel exactly once
    out.view(-1, 3).index_copy_(0, B["dst"], recv.index_select(0, B["src"]))
    return out


def communicator(rank, world, group=None, device=None):
    """The process's librtamd communicator for `group` (rt_comm_create), made once: rank 0's
    rt_comm_unique_id is broadcast over the group, then every rank joins."""
    import torch
    import torch.distributed as dist
    key = (id(group), rank, world)
    if key not in _comms:
        dev = device if device is not None else torch.device("cuda", torch.cuda.current_device())
        buf = torch.zeros(gpu._lib.RT_COMM_ID_BYTES, dtype=torch.uint8, device=dev)
        if rank == 0:
            buf.copy_(torch.frombuffer(bytearray(gpu.comm_unique_id()), dtype=torch.uint8))
        dist.broadcast(buf, src=0, group=group)
        ctx = gpu.default_context(dev.index if getattr(dev, "index", None) is not None else 0)
        _comms[key] = gpu.Comm(bytes(buf.cpu().numpy().tobytes()), rank, world, ctx=ctx)
    return _comms[key]


def render_frame(scene, nx, ny, spp_begin, spp_count, seed, rank, world, local=None, frame=None, stream=None,
                 ctx=None):
    """One frame's passes on this rank's GPU.  world == 1: straight into `frame`
    (a full-frame device tensor).  world > 1: this rank's tiles into `local`
    (compact, 3 x shard pixels, zeroed by the caller), then gather_frame;
    returns the frame (``frame`` if given) on rank 0 and None elsewhere."""
    if stream is None:                          # order after the caller's torch work (e.g. zeroing the buffers)
        import torch
        stream = torch.cuda.current_stream().cuda_stream
    if world == 1:
        gpu.render_device(scene, nx, ny, spp_begin, spp_count, seed, frame.data_ptr(), stream=stream, ctx=ctx)
        return frame
    gpu.render_shard_device(scene, nx, ny, spp_begin, spp_count, seed, rank, world, local.data_ptr(), stream=stream,
                            ctx=ctx)
    return gather_frame(local, nx, ny, rank, world, out=frame)


def local_size(nx, ny, rank, world):
    """Values in rank's compact accumulator (3 x its pixel count)."""
    return 3 * len(shard_pixels(nx, ny, world)[rank])
