"""The multi-process frame on the GPU: two ranks (gloo process group, both on
cuda:0 — the one-GPU box has no second device for RCCL) each render their
interleaved tiles with librtamd (rt_render_shard_device, compact accumulator)
through rtamd.dist.render_frame — bench.py's per-step call — and rank 0's
gathered frame must equal a one-process rt_render_device frame bit for bit.
Only the transport differs from the 8-GPU bench (gloo through host memory
instead of RCCL over xGMI); the RCCL path itself — rt_gather_shards behind
the C ABI — runs at world size 1 (test_rccl_gather_world1_equals_render_device,
test_capi_gather_shards_world1)."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu

NX, NY, SPP, SEED = 96, 54, 3, 0x5EED0002


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, out_path, wavefront):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "scheme-raytrace_amd"))
    import torch
    import torch.distributed as dist

    from rtamd import dist as rdist
    from rtamd import gpu, scenes

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    torch.cuda.set_device(0)
    scene = scenes.random_scene(NX, NY)
    ctx = gpu.default_context(0)
    if wavefront:                                # the wavefront kernels, not only the tail kernel
        ctx.set_option("tail_off", 1)
    local = torch.zeros(rdist.local_size(NX, NY, rank, world), dtype=torch.float64, device="cuda")
    frame = rdist.render_frame(scene, NX, NY, 0, SPP, SEED, rank, world, local=local, ctx=ctx)
    torch.cuda.synchronize()
    if rank == 0:
        np.save(out_path, frame.cpu().numpy())
    else:
        assert frame is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,wavefront", [(2, True), (3, False)])
def test_multiprocess_tile_shards_equal_one_process_frame(sched, tmp_path, monkeypatch, world, wavefront):
    import torch
    from rtamd import gpu, scenes
    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(world, _free_port(), out, wavefront), nprocs=world, join=True)
    if wavefront:
        sched.set_option("tail_off", 1)
    full = torch.zeros(NX * NY * 3, dtype=torch.float64, device="cuda")
    gpu.render_device(scenes.random_scene(NX, NY), NX, NY, 0, SPP, SEED, full.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(np.load(out), full.cpu().numpy())


def _nccl_worker(rank, world, port, out_path):
    """RCCL ("nccl" backend) at world size 1 on cuda:0 — the only RCCL
    configuration a one-GPU box can run: the rank renders its (only) shard
    into a compact device accumulator and rtamd.dist.gather_frame moves it
    over RCCL into a device frame — through the C ABI since round 5
    (rt_comm_create with the id broadcast over the process group, then
    rt_gather_shards) — twice (the second frame reuses the communicator and
    the cached pixel lists)."""
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, os.path.join(root, "scheme-raytrace_amd"))
    import torch
    import torch.distributed as dist

    from rtamd import dist as rdist
    from rtamd import gpu, scenes

    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=rank, world_size=world, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl"
    scene = scenes.random_scene(NX, NY)
    ctx = gpu.default_context(0)
    local = torch.zeros(rdist.local_size(NX, NY, rank, world), dtype=torch.float64, device="cuda")
    frame = torch.full((NX * NY * 3,), -1.0, dtype=torch.float64, device="cuda")
    frames = []
    for _ in range(2):
        local.zero_()
        gpu.render_shard_device(scene, NX, NY, 0, SPP, SEED, rank, world, local.data_ptr(),
                                stream=torch.cuda.current_stream().cuda_stream, ctx=ctx)
        out = rdist.gather_frame(local, NX, NY, rank, world, out=frame)
        assert out is frame and out.device.type == "cuda"
        frames.append(out.cpu().numpy().copy())
    torch.cuda.synchronize()
    assert np.array_equal(frames[0], frames[1])
    np.save(out_path, frames[0])
    dist.barrier()
    dist.destroy_process_group()


def test_rccl_gather_world1_equals_render_device(sched, tmp_path):
    import torch
    from rtamd import gpu, scenes
    out = str(tmp_path / "frame.npy")
    mp.spawn(_nccl_worker, args=(1, _free_port(), out), nprocs=1, join=True)
    full = torch.zeros(NX * NY * 3, dtype=torch.float64, device="cuda")
    gpu.render_device(scenes.random_scene(NX, NY), NX, NY, 0, SPP, SEED, full.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(np.load(out), full.cpu().numpy())


def test_capi_gather_shards_world1(sched):
    """The frame-end gather behind the C ABI alone (rt_comm_unique_id, rt_comm_create, rt_gather_shards,
    rt_comm_destroy — what a Scheme or C host calls), without torch.distributed: world size 1, the rank's
    compact accumulator into a device frame, bitwise equal to rt_render_device; two frame sizes on one
    communicator (the pixel lists are rebuilt when the size changes)."""
    import torch
    from rtamd import dist as rdist
    from rtamd import gpu, scenes
    comm = gpu.Comm(gpu.comm_unique_id(), 0, 1, ctx=sched)
    try:
        for nx, ny in ((NX, NY), (53, 37)):
            scene = scenes.random_scene(nx, ny)
            full = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
            gpu.render_device(scene, nx, ny, 0, SPP, SEED, full.data_ptr(), ctx=sched)
            local = torch.zeros(rdist.local_size(nx, ny, 0, 1), dtype=torch.float64, device="cuda")
            gpu.render_shard_device(scene, nx, ny, 0, SPP, SEED, 0, 1, local.data_ptr(), ctx=sched)
            frame = torch.full((nx * ny * 3,), -1.0, dtype=torch.float64, device="cuda")
            torch.cuda.synchronize()
            comm.gather_shards(nx, ny, local.data_ptr(), frame.data_ptr())
            assert torch.equal(frame, full)
    finally:
        comm.close()


def test_bench_two_ranks_self_verifying(tmp_path):
    """bench.py at N=2 under torch.distributed.run (gloo rehearsal: both ranks
    on cuda:0), launched as a fresh child process: the JSON line reports
    n_gpus 2, per-rank timings, and both parity legs — a band re-rendered on
    rank 0 and rows of the gathered frame itself — pass against the oracle.
    This is the line the driver's 8-GPU SCALE run prints at every N."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, RTAMD_DIST_BACKEND="gloo", OMP_NUM_THREADS=os.environ.get("OMP_NUM_THREADS", "8"))
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"),
           "--gpus", "2", "--steps", "1", "--warmup", "0", "--spp", "8", "--nx", "320", "--ny", "180",
           "--cpu-baseline-seconds", "2"]
    r = subprocess.run(cmd, cwd=root, env=env, capture_output=True, text=True, timeout=240)
    assert r.returncode == 0, r.stderr[-4000:]
    lines = [l for l in r.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1, r.stdout[-2000:]
    d = json.loads(lines[0])
    print(json.dumps({k: d[k] for k in ("value", "n_gpus", "per_rank_ms_per_step")}),
          d["parity"]["rms_vs_oracle"], d["parity_frame"]["rms_vs_oracle"], d["parity_frame"]["rows"])
    assert d["n_gpus"] == 2 and d["config"]["parallelism"].startswith("tile-shard2")
    assert d["cpu_baseline"] is None                        # an N = 1 figure only
    assert d["parity"]["pass"] and d["parity_frame"]["pass"]
    assert d["parity_frame"]["pixels_gt_1e-9"] <= max(2, d["parity_frame"]["pixels"] // 200)
    assert d["per_rank_ms_per_step"]["render_max"] >= d["per_rank_ms_per_step"]["render_min"] > 0


@pytest.mark.parametrize("world", [3, 8])
def test_gather_shards_local_world_n_equals_render_device(sched, world):
    """rt_gather_shards' N > 1 receive layout and placement, executed on one GPU (round 6; RCCL cannot put
    two ranks on one device): every shard of `world` rendered into its own compact accumulator
    (rt_render_shard_device), then rt_gather_shards_local — the shared gather plan (rt_gather_layout's
    counts / offsets, rank 0's receive buffer at 3 * (off[r] - count[0])) and placement kernel, with device
    copies standing in for ncclRecv — must give rt_render_device's frame bit for bit, at world 3 (tile
    stride 5) and 8, on a frame whose edge tiles are partial."""
    import torch
    from rtamd import gpu, scenes
    nx, ny, spp = 200, 120, 3
    scene = scenes.random_scene(nx, ny)
    cnt, off = gpu.gather_layout(nx, ny, world)
    shards = [torch.zeros(3 * int(c), dtype=torch.float64, device="cuda") for c in cnt]
    frame = torch.full((nx * ny * 3,), -1.0, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()                             # torch's fills before the library's stream
    for r, buf in enumerate(shards):
        gpu.render_shard_device(scene, nx, ny, 0, spp, SEED, r, world, buf.data_ptr())
    gpu.gather_shards_local(nx, ny, [b.data_ptr() for b in shards], frame.data_ptr())
    full = torch.zeros(nx * ny * 3, dtype=torch.float64, device="cuda")
    torch.cuda.synchronize()
    gpu.render_device(scene, nx, ny, 0, spp, SEED, full.data_ptr())
    torch.cuda.synchronize()
    got, want = frame.cpu().numpy(), full.cpu().numpy()
    assert (got >= 0).all()                              # every pixel was placed
    assert np.array_equal(got, want)
    # a second frame size on the same context rebuilds the plan
    nx2, ny2 = 64, 40
    sc2 = scenes.random_scene(nx2, ny2)
    cnt2, _ = gpu.gather_layout(nx2, ny2, world)
    sh2 = [torch.zeros(3 * int(c), dtype=torch.float64, device="cuda") for c in cnt2]
    torch.cuda.synchronize()
    for r, b in enumerate(sh2):
        gpu.render_shard_device(sc2, nx2, ny2, 0, 1, SEED, r, world, b.data_ptr())
    f2 = torch.zeros(nx2 * ny2 * 3, dtype=torch.float64, device="cuda")
    w2 = torch.zeros_like(f2)
    torch.cuda.synchronize()
    gpu.gather_shards_local(nx2, ny2, [b.data_ptr() for b in sh2], f2.data_ptr())
    gpu.render_device(sc2, nx2, ny2, 0, 1, SEED, w2.data_ptr())
    torch.cuda.synchronize()
    assert np.array_equal(f2.cpu().numpy(), w2.cpu().numpy())
