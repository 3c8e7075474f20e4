"""The multi-rank path on CPU (gloo): row sharding, the gather to rank 0 and the reorder
reproduce the single-process frame exactly, for 2 and 3 ranks.

On the GPU each rank's slab comes from rt_launch(shard=rank, nshards=world); here the
test renders each rank's slab rows with the oracle (test-side stand-in for the kernel)
so the host logic — eraytracer_amd.dist.shard_global_rows / gather_frame / unshard — runs
unchanged over a real torch.distributed process group."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from eraytracer_amd import _native as N
from eraytracer_amd import scenes
from eraytracer_amd.dist import gather_frame, shard_global_rows, shard_rows, unshard

W, H, D, RB = 40, 37, 4, 4


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import oracle as O
    el = N.marshal(scenes.s64())
    g = shard_global_rows(H, RB, world, rank)
    slab = np.zeros((len(g), W, 3))
    for i, row in enumerate(g):
        if row >= 0:
            slab[i] = O.render(el, W, H, D, mode=O.MEMO, row0=int(row), nrows=1, threads=1)[0]
    frame = gather_frame(torch.from_numpy(slab), H, RB, world, rank)
    if rank == 0:
        np.save(out_path, frame.numpy())
    else:
        assert frame is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_gather_reassembles_frame(tmp_path, oracle, world):
    out = str(tmp_path / "frame.npy")
    mp.spawn(_worker, args=(world, _free_port(), out), nprocs=world, join=True)
    frame = np.load(out)
    ref = oracle.render(N.marshal(scenes.s64()), W, H, D, mode=oracle.MEMO)
    assert frame.shape == ref.shape
    assert np.array_equal(frame.view(np.int64), ref.view(np.int64))


def test_unshard_is_inverse_of_sharding():
    for h, rb, ns in [(37, 4, 3), (64, 16, 4), (5, 16, 8), (100, 7, 1)]:
        rows = shard_rows(h, rb, ns)
        img = torch.arange(h * 2).reshape(h, 2)
        slabs = torch.full((ns, rows, 2), -1, dtype=img.dtype)
        seen = []
        for s in range(ns):
            g = shard_global_rows(h, rb, ns, s)
            for i, row in enumerate(g):
                if row >= 0:
                    slabs[s, i] = img[row]
                    seen.append(int(row))
        assert sorted(seen) == list(range(h))  # every row owned by exactly one shard
        assert torch.equal(unshard(slabs, h, rb), img)


def _pipe_worker(rank, world, port, out_path, nframes):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eraytracer_amd.dist import SlabPipeline
    rows = shard_rows(H, RB, world)
    g = torch.from_numpy(shard_global_rows(H, RB, world, rank))
    slabs = [torch.zeros((rows, W)), torch.zeros((rows, W))]
    gbufs = [torch.zeros((world, rows, W)), torch.zeros((world, rows, W))] if rank == 0 else None
    pipe = SlabPipeline(world, rank, slabs, gbufs, lambda gb: unshard(gb, H, RB).clone())
    frames = []
    for f in range(nframes):
        # "render" frame f: every pixel of global row r holds f*1000 + r (padding rows -1)
        pipe.slab.copy_(torch.where(g[:, None] >= 0, f * 1000.0 + g[:, None].double(), -1.0).float().expand(rows, W))
        out = pipe.submit()
        if out is not None:
            frames.append(out)
    out = pipe.drain()
    if out is not None:
        frames.append(out)
    if rank == 0:
        np.save(out_path, torch.stack(frames).numpy())
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_pipelined_gather_frames_in_order(tmp_path, world):
    """SlabPipeline (bench.py's multi-GPU step): frame i+1 renders while frame i is gathered;
    rank 0 must still get every frame, complete, in order and in row order."""
    out = str(tmp_path / "frames.npy")
    nframes = 5
    mp.spawn(_pipe_worker, args=(world, _free_port(), out, nframes), nprocs=world, join=True)
    frames = np.load(out)
    assert frames.shape == (nframes, H, W)
    for f in range(nframes):
        expect = (f * 1000.0 + np.arange(H, dtype=np.float64))[:, None] * np.ones((1, W))
        assert np.array_equal(frames[f], expect.astype(np.float32)), f"frame {f}"


# ---- compact gather (dist.CompactGather, bench.py's default for world > 1) ----------------
def _expected_frame(frame_no):
    """Frame `frame_no`: pixel (x, r) holds a value when (x + r + frame_no) % 3 == 0, else the
    background +0.0 — except pixel (1, 1), which holds (0, -0.0, 0): non-zero bits, so sent."""
    g = torch.arange(H)
    x = torch.arange(W)
    val = (frame_no * 1000.0 + g[:, None] * 10.0 + x[None, :] / 64.0).float()
    keep = (x[None, :] + g[:, None] + frame_no) % 3 == 0
    z = torch.zeros(())
    f = torch.stack([torch.where(keep, val, z), torch.where(keep, -val, z), torch.where(keep, val * 0.5, z)], -1)
    if not keep[1, 1]:
        f[1, 1, 1] = -0.0
    return f


def _sparse_slab(frame_no, rank, world, rows):
    """`rank`'s slab of that frame; padding rows past the image hold garbage (never read)."""
    g = torch.from_numpy(shard_global_rows(H, RB, world, rank))
    slab = torch.full((rows, W, 3), 7.0)
    ok = g >= 0
    slab[ok] = _expected_frame(frame_no)[g[ok]]
    return slab


def _compact_worker(rank, world, port, out_path, nframes):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eraytracer_amd.dist import CompactGather
    from tests.slab_ref import RefCodec
    rows = shard_rows(H, RB, world)
    codec = RefCodec(W, H, RB, world)
    frame = torch.empty((H, W, 3), dtype=torch.float32) if rank == 0 else None
    cg = CompactGather(codec, world, rank, rows * W * 3, torch.float32, "cpu", frame)
    frames = []
    for f in range(nframes):
        out = cg.submit(_sparse_slab(f, rank, world, rows), rank)
        if out is not None:
            frames.append(out.clone())
    cg.drain(on_frame=lambda fr: frames.append(fr.clone()))
    if rank == 0:
        np.save(out_path, torch.stack(frames).numpy())
    else:
        assert not frames
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_gloo_compact_gather_frames_in_order(tmp_path, world):
    """CompactGather: headers gathered, exact value counts sent point-to-point, decoded on
    rank 0, frames two deep in flight: every frame arrives complete, exact and in order."""
    out = str(tmp_path / "frames.npy")
    nframes = 6
    mp.spawn(_compact_worker, args=(world, _free_port(), out, nframes), nprocs=world, join=True)
    frames = np.load(out)
    assert frames.shape == (nframes, H, W, 3)
    for f in range(nframes):
        assert np.array_equal(frames[f].view(np.int32), _expected_frame(f).numpy().view(np.int32)), f"frame {f}"


def test_ref_codec_round_trip_and_layout():
    from tests.slab_ref import RefCodec
    for world in (1, 2, 3):
        codec = RefCodec(W, H, RB, world)
        rows = shard_rows(H, RB, world)
        hdrs, vals = [], []
        for s in range(world):
            slab = _sparse_slab(2, s, world, rows)
            h = torch.empty(codec.header_bytes, dtype=torch.uint8)
            v = torch.full((rows * W * 3,), float("nan"))
            codec.pack(slab, s, h, v)
            n = int(h[:8].view(torch.int64)[0])
            assert n == int(((slab.view(torch.int32) != 0).any(-1) & (torch.from_numpy(
                shard_global_rows(H, RB, world, s)) >= 0)[:, None]).sum())
            hdrs.append(h)
            vals.append(v)
        frame = torch.empty((H, W, 3))
        codec.unpack(hdrs, vals, frame)
        assert torch.equal(frame.view(torch.int32), _expected_frame(2).view(torch.int32))


def _verify_worker(rank, world, port, out_path, corrupt, first=0):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eraytracer_amd.dist import CompactGather, verify_compact_gather
    from tests.slab_ref import RefCodec
    ns, shard = world - first, max(rank - first, 0)  # first = 1: rank 0 assembles
    rows = shard_rows(H, RB, ns)
    codec = RefCodec(W, H, RB, ns)
    frame = torch.empty((H, W, 3), dtype=torch.float32) if rank == 0 else None
    cg = CompactGather(codec, world, rank, rows * W * 3, torch.float32, "cpu", frame, first=first)

    def make_slab(i):
        if first and rank == 0:
            return None
        s = _sparse_slab(i, shard, ns, rows)
        if corrupt and rank == world - 1 and i == 1:
            s[0, 3] = 42.0  # one wrong pixel on the last rank
        return s

    try:
        n = verify_compact_gather(cg, make_slab, _expected_frame, rank, nframes=3, shard=shard)
        res = f"ok {n}"
    except RuntimeError as e:
        res = f"error {e}"
    if rank == 0:
        with open(out_path, "w") as f:
            f.write(res)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,corrupt,first", [(2, False, 0), (3, False, 0), (3, True, 0), (3, False, 1),
                                                (4, True, 1)])
def test_gloo_bench_self_check(tmp_path, world, corrupt, first):
    """bench.py --gpus N's check before timing (dist.verify_compact_gather): the compact gather's
    frames equal the one-shard frames, and a single wrong pixel on any rank is caught — also with
    an assembling rank 0 (first = 1)."""
    out = str(tmp_path / "res.txt")
    mp.spawn(_verify_worker, args=(world, _free_port(), out, corrupt, first), nprocs=world, join=True)
    res = open(out).read()
    if corrupt:
        assert res.startswith("error") and "frame 1" in res and "1 pixels" in res, res
    else:
        assert res == "ok 3", res


def _assemble_worker(rank, world, port, out_path, nframes):
    """CompactGather with an assembling rank 0: ranks 1 .. world-1 render shards 0 .. world-2 of
    world-1; rank 0 submits nothing and decodes."""
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from eraytracer_amd.dist import CompactGather
    from tests.slab_ref import RefCodec
    ns = world - 1
    rows = shard_rows(H, RB, ns)
    codec = RefCodec(W, H, RB, ns)
    frame = torch.empty((H, W, 3), dtype=torch.float32) if rank == 0 else None
    cg = CompactGather(codec, world, rank, rows * W * 3, torch.float32, "cpu", frame, first=1)
    frames = []
    for f in range(nframes):
        slab = None if rank == 0 else _sparse_slab(f, rank - 1, ns, rows)
        out = cg.submit(slab, max(rank - 1, 0))
        if out is not None:
            frames.append(out.clone())
    cg.drain(on_frame=lambda fr: frames.append(fr.clone()))
    if rank == 0:
        np.save(out_path, torch.stack(frames).numpy())
    else:
        assert not frames
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3, 4])
def test_gloo_compact_gather_with_assembling_rank0(tmp_path, world):
    """bench.py --rank0 assemble (the default from 4 ranks): rank 0 renders no rows, the other ranks'
    shards arrive complete, exact and in order."""
    out = str(tmp_path / "frames.npy")
    nframes = 6
    mp.spawn(_assemble_worker, args=(world, _free_port(), out, nframes), nprocs=world, join=True)
    frames = np.load(out)
    assert frames.shape == (nframes, H, W, 3)
    for f in range(nframes):
        assert np.array_equal(frames[f].view(np.int32), _expected_frame(f).numpy().view(np.int32)), f"frame {f}"


def test_assembling_rank0_must_submit_nothing():
    from eraytracer_amd.dist import CompactGather
    from tests.slab_ref import RefCodec
    with pytest.raises(ValueError):
        CompactGather(RefCodec(W, H, RB, 1), 1, 0, 10, torch.float32, "cpu", None, first=1)
