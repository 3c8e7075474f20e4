"""Multi-GPU frame rendering: one process per GPU, rows sharded, one gather to rank 0.

The reference's distributed strategy (raytraced_pixel_list_distributed/4,
raytracer.erl:121-149) splits the pixels into ~64 chunks spawned on pool nodes, every
worker sends one message per pixel to a master (:169-178), and the master returns the
whole list to the caller.  Here the frame's rows are dealt to ranks in interleaved
blocks of ``row_block`` rows (sky rows and floor rows cost differently, so contiguous
halves would be unbalanced); every rank renders its rows into one contiguous slab on its
own GPU; the slabs are gathered to rank 0 with a single collective (RCCL over xGMI for
the ``nccl`` backend) and rank 0 puts the rows back in image order.  That gather is the
path's only exchange step — the reference's master collecting the pixel list.
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native as N

PRECISIONS = {"f64": N.RT_OUT_F64, "f32": N.RT_OUT_F32}
ORDERS = {"exact": N.RT_ORDER_EXACT, "fast": N.RT_ORDER_FAST}


def shard_rows(height: int, row_block: int, nshards: int) -> int:
    """Rows in every shard's slab (rt_shard_rows): whole row blocks, equal for all shards."""
    span = row_block * nshards
    return -(-height // span) * row_block


def shard_global_rows(height: int, row_block: int, nshards: int, shard: int) -> np.ndarray:
    """Global row of each slab row of `shard` (-1 for padding past the image)."""
    rows = shard_rows(height, row_block, nshards)
    local = np.arange(rows)
    g = ((local // row_block) * nshards + shard) * row_block + local % row_block
    return np.where(g < height, g, -1)


def unshard(gathered, height: int, row_block: int):
    """Reassemble gathered slabs ``[nshards, slab_rows, ...]`` into ``[height, ...]`` (torch,
    any device): slab block b of shard s holds global rows ``(b*nshards + s)*row_block + i``."""
    ns, rows = gathered.shape[0], gathered.shape[1]
    nb = rows // row_block
    rest = tuple(gathered.shape[2:])
    x = gathered.reshape((ns, nb, row_block) + rest).transpose(0, 1)  # [nb, ns, rb, ...]
    return x.reshape((nb * ns * row_block,) + rest)[:height]


def gather_frame(slab, height: int, row_block: int, world: int, rank: int, group=None, out=None, gather_buf=None):
    """Collect every rank's slab on rank 0 and return the full frame there (None elsewhere)."""
    import torch
    import torch.distributed as dist
    if world == 1:
        return slab[:height]
    if rank == 0:
        if gather_buf is None:
            gather_buf = torch.empty((world,) + tuple(slab.shape), dtype=slab.dtype, device=slab.device)
        dist.gather(slab, gather_list=list(gather_buf.unbind(0)), dst=0, group=group)
        frame = unshard(gather_buf, height, row_block)
        if out is not None:
            out.copy_(frame)
            return out
        return frame
    dist.gather(slab, gather_list=None, dst=0, group=group)
    return None


class SlabPipeline:
    """Double-buffered gather of per-rank slabs: frame i's gather runs (async, on the
    collective's own stream) while frame i+1 renders into the other slab; rank 0 reorders a
    frame when its gather is complete.

    ``slabs`` are this rank's two slab buffers, ``gbufs`` rank 0's two [world, rows, ...]
    gather buffers (None elsewhere), ``reorder(gbuf)`` rank 0's reassembly into the frame.
    Stream order keeps it safe: frame i+2 renders into frame i's slab only after frame i's
    gather has been waited on, and gathers into frame i's buffer only after its reorder."""

    def __init__(self, world, rank, slabs, gbufs=None, reorder=None, group=None):
        self.world, self.rank, self.group = world, rank, group
        self.slabs, self.gbufs, self.reorder = slabs, gbufs, reorder
        self.i = 0            # frames started
        self.pending = []     # (work, buffer index) in flight

    @property
    def slab(self):
        """The slab the next frame renders into."""
        return self.slabs[self.i % 2]

    def submit(self):
        """Start gathering the frame just rendered into ``slab``; finish the previous one."""
        import torch.distributed as dist
        b = self.i % 2
        self.i += 1
        if self.world == 1:
            return self.slabs[b]
        gl = list(self.gbufs[b].unbind(0)) if self.rank == 0 else None
        work = dist.gather(self.slabs[b], gather_list=gl, dst=0, group=self.group, async_op=True)
        self.pending.append((work, b))
        return self.complete() if len(self.pending) > 1 else None

    def complete(self):
        """Wait for the oldest gather in flight and reorder it (rank 0: returns the frame)."""
        work, b = self.pending.pop(0)
        work.wait()
        if self.rank == 0:
            return self.reorder(self.gbufs[b])
        return None

    def drain(self):
        out = None
        while self.pending:
            out = self.complete()
        return out


class SlabCodec:
    """The HIP slab codec of the compact gather (rt_slab_pack / rt_slab_unpack,
    include/rt_mi355x.h "compact slab transfer"): a slab becomes a fixed-size header (count,
    per-256-pixel offsets, one bit per pixel) plus the non-background pixels' values; rank 0
    decodes every shard straight into the row-major frame (rt_unshard fused with the decode).
    Device tensors only: there is no host implementation in the product."""

    def __init__(self, width: int, height: int, row_block: int, world: int, precision: str):
        self.L = N.lib()
        self.w, self.h, self.rb, self.world = width, height, row_block, world
        self.prec = PRECISIONS[precision]
        self.header_bytes = int(self.L.rt_slab_header_bytes(width, height, row_block, world))
        if self.header_bytes == 0:
            raise ValueError("rt_slab_header_bytes: bad frame arguments")

    @staticmethod
    def _stream(t):
        import torch
        return torch.cuda.current_stream(t.device).cuda_stream

    def pack(self, slab, shard, header, values):
        N.check(self.L.rt_slab_pack(slab.data_ptr(), self.w, self.h, self.rb, shard, self.world, self.prec,
                                    header.data_ptr(), values.data_ptr(), self._stream(slab)), "rt_slab_pack")

    def unpack(self, headers, values, frame):
        n = len(headers)
        hp = (ctypes.c_void_p * n)(*[h.data_ptr() for h in headers])
        vp = (ctypes.c_void_p * n)(*[v.data_ptr() for v in values])
        N.check(self.L.rt_slab_unpack(hp, vp, self.w, self.h, self.rb, n, self.prec, frame.data_ptr(),
                                      self._stream(frame)), "rt_slab_unpack")


class CompactGather:
    """Pipelined compact gather of per-rank slabs to rank 0 (the default for world > 1).

    Per frame i, on every rank: ``codec.pack`` encodes the slab just rendered (same stream);
    the fixed-size headers are gathered to rank 0 (one collective), which also tells rank 0
    every shard's value count; then each rank sends exactly its non-background values to
    rank 0 (grouped point-to-point, RCCL over xGMI), and rank 0 decodes all shards into the
    frame.  The exchange runs on a side stream, behind the render: ``submit(i)`` issues frame
    i's header gather and the copy of its counts to pinned host memory (an event marks the
    copy), frame i-2's value transfer (its counts read on the host after waiting for that copy
    event alone — two frames later it has normally long fired, so the host does not stall, and
    no other work on the side stream is waited for) and frame i-3's decode, which it returns on
    rank 0 (complete once ``frame_ready`` has fired: the decode runs on the side stream, beside
    the next render).  ``drain()`` finishes the frames in flight.  The order of collectives is
    the same on every rank (it depends only on the frame count, never on timing).

    Buffers form a ring of four frames.  Frame i's pack waits for the event that ends frame
    i-4's send (rank 0: its decode), so the caller may render consecutive frames on different
    streams; every collective is issued on the side stream behind an event of the pack it
    reads, so it never waits for a later render.

    ``first`` = 1: rank 0 renders no rows and only assembles (the codec's shards are ranks 1 ..
    world-1, shard = rank - 1); it submits None and its header in the gather is ignored.
    """

    RING = 4
    LAG = 2  # frames between a frame's header gather and its value transfer

    def __init__(self, codec, world, rank, slab_elems, dtype, device, frame, group=None, first=0):
        import torch
        self.torch = torch
        self.codec, self.world, self.rank, self.group = codec, world, rank, group
        if first not in (0, 1) or (first == 1 and world < 2):
            raise ValueError("first: 0 (every rank renders) or 1 (rank 0 assembles; world >= 2)")
        self.first = first
        self.frame = frame
        self.cuda = torch.device(device).type == "cuda"
        hb = codec.header_bytes
        mk = lambda *shape, dt: torch.empty(shape, dtype=dt, device=device)  # noqa: E731
        self.hdr = [torch.zeros(hb, dtype=torch.uint8, device=device) for _ in range(self.RING)]
        self.vals = [mk(slab_elems, dt=dtype) for _ in range(self.RING)]
        self.ghdr = self.gvals = None
        if rank == 0:
            self.ghdr = [mk(world, hb, dt=torch.uint8) for _ in range(self.RING)]
            self.gvals = [mk(world, slab_elems, dt=dtype) for _ in range(self.RING)]
        self.xs = torch.cuda.Stream(device) if self.cuda else None
        self.counts = [torch.zeros(world, dtype=torch.int64, pin_memory=self.cuda) for _ in range(self.RING)]
        self.i = 0
        self.free = [None] * self.RING      # event: the slot's last send (decode on rank 0) is done
        self.frame_ready = None             # rank 0: the last returned frame is complete after this
        self.headed = []   # (ring slot, event of its counts' copy to the host)
        self.moving = []   # (ring slot, value transfer works)

    def _side(self):
        import contextlib
        return self.torch.cuda.stream(self.xs) if self.cuda else contextlib.nullcontext()

    def submit(self, slab, shard):
        """Hand over the slab of this rank's shard `shard` just rendered (None on an assembling
        rank 0, which renders nothing)."""
        torch = self.torch
        b = self.i % self.RING
        self.i += 1
        if self.free[b] is not None:  # slot b's last send / decode has read its buffers
            torch.cuda.current_stream().wait_event(self.free[b])
            self.free[b] = None
        if slab is not None:
            self.codec.pack(slab, shard, self.hdr[b], self.vals[b])
        elif not (self.first == 1 and self.rank == 0):
            raise ValueError("only an assembling rank 0 submits no slab")
        ev = None
        if self.cuda:
            ev = torch.cuda.Event()
            ev.record()
        out = None
        if len(self.headed) >= self.LAG:
            self._send(*self.headed.pop(0))
        if len(self.moving) > 1:
            out = self._finish(*self.moving.pop(0))
        self._gather_headers(b, ev)
        return out

    def drain(self, on_frame=None):
        """Finish every frame in flight (oldest first); ``on_frame(frame)`` sees each decoded
        frame on rank 0 before the next one overwrites it.  Returns the last."""
        out = None
        while self.headed or self.moving:
            if self.headed:
                self._send(*self.headed.pop(0))
            out = self._finish(*self.moving.pop(0))
            if out is not None and on_frame is not None:
                on_frame(out)
        return out

    def _gather_headers(self, b, ev):
        """Frame slot b: gather the headers to rank 0, then copy the value counts (the first
        8 bytes of each header) to pinned host memory; the copy's event is kept for _send."""
        torch = self.torch
        import torch.distributed as dist
        with self._side():
            if ev is not None:
                self.xs.wait_event(ev)
            gl = list(self.ghdr[b].unbind(0)) if self.rank == 0 else None
            w = dist.gather(self.hdr[b], gather_list=gl, dst=0, group=self.group, async_op=True)
            w.wait()  # RCCL: the side stream waits for the gather (gloo: the host does)
            src = self.ghdr[b][:, :8] if self.rank == 0 else self.hdr[b][:8].unsqueeze(0)
            cnt = src.contiguous().view(torch.int64).flatten()
            self.counts[b][: cnt.numel()].copy_(cnt, non_blocking=self.cuda)
            cev = None
            if self.cuda:
                cev = torch.cuda.Event()
                cev.record()
        self.headed.append((b, cev))

    def _send(self, b, cev):
        """Frame in slot b: read its counts on the host, then send the values to rank 0.  The
        host waits for the counts' copy event, which the side stream orders after its earlier
        work as well (older frames' decode and transfer waits): by then, with frames in flight,
        those are normally done."""
        import torch.distributed as dist
        with self._side():
            if cev is not None:
                cev.synchronize()
            counts = [int(c) for c in self.counts[b].tolist()]
            # at least one pixel per message: every rank takes part in every batch
            n = [max(c, 1) * 3 for c in counts]
            ops = []
            if self.rank == 0:
                for s in range(1, self.world):
                    ops.append(dist.P2POp(dist.irecv, self.gvals[b][s][: n[s]], s, group=self.group))
            else:
                ops.append(dist.P2POp(dist.isend, self.vals[b][: n[0]], 0, group=self.group))
            works = dist.batch_isend_irecv(ops) if ops else []  # a one-rank group sends nothing
        self.moving.append((b, works))

    def _finish(self, b, works):
        """Wait (on the side stream) for frame slot b's transfer; rank 0 then decodes it there,
        beside the next render (the decode is HBM-bound, the render FP64-bound).  The event
        ``free[b]`` marks slot b's buffers reusable; on rank 0 ``frame_ready`` marks the frame
        complete."""
        with self._side():
            for w in works:
                w.wait()
            if self.rank == 0:  # the rendering ranks' shards: ranks first .. world-1
                vals = ([self.vals[b]] if self.first == 0 else []) + [self.gvals[b][s] for s in range(1, self.world)]
                self.codec.unpack(list(self.ghdr[b].unbind(0))[self.first:], vals, self.frame)
            if self.cuda:
                ev = self.torch.cuda.Event()
                ev.record()
                self.free[b] = ev
                if self.rank == 0:
                    self.frame_ready = ev
        return self.frame if self.rank == 0 else None


def verify_compact_gather(cg, make_slab, reference, rank, nframes=2, shard=None):
    """The multi-rank bench's self-check before timing: every rank renders its slab of a check
    frame (``make_slab(i)``, frame i; None on an assembling rank 0), the slabs go through the
    compact gather ``cg`` exactly as in the timed loop (frames in flight), and rank 0 compares
    every reassembled frame bit for bit with ``reference(i)`` (a one-shard render of the same
    frame).  ``shard``: this rank's shard (default: its rank).  Raises on a mismatch; returns the
    number of frames checked on rank 0 (0 elsewhere)."""
    shard = rank if shard is None else shard
    import torch
    got = []

    def keep(f):
        if cg.frame_ready is not None:
            torch.cuda.current_stream().wait_event(cg.frame_ready)
        got.append(f.clone())
        if cg.cuda:
            torch.cuda.synchronize()

    for i in range(nframes):
        out = cg.submit(make_slab(i), shard)
        if out is not None:
            keep(out)
    cg.drain(on_frame=keep)
    if rank != 0:
        return 0
    if len(got) != nframes:
        raise RuntimeError(f"compact gather returned {len(got)} of {nframes} frames")
    for i, f in enumerate(got):
        ref = reference(i)
        a = f.contiguous().view(torch.int32 if f.dtype == torch.float32 else torch.int64)
        b = ref.to(f.device).contiguous().view(a.dtype)
        if not torch.equal(a, b):
            bad = int((a != b).any(-1).sum())
            raise RuntimeError(f"gathered frame {i} differs from the one-shard frame in {bad} pixels")
    return nframes


class FrameRenderer:
    """Renders this rank's rows of a W x H frame on its GPU and gathers the frame to rank 0.

    ``step()`` = one pass of the hot path over one frame: the render kernel on this
    rank's rows (rt_launch) and, for world > 1, the gather plus rank 0's reorder
    (rt_unshard, two strided device copies).

    ``inflight`` > 1 keeps that many frames in flight: one render context (rt_prepare:
    its own work space), slab and HIP stream per slot, frames dealt to the slots in turn.  A
    frame's reflection chain ends in a latency-bound tail (sparse deep levels, the chain
    walk); the next frames' dense primary and shading kernels fill it.  Each context then
    runs its kernels on its slot's stream alone (RT_CFG_SIDE_STREAMS = 0), so the process
    stays within its hardware queues.  ``stream`` is the stream of the last launched frame;
    work on that frame (the gather's pack) goes on it.  ``cull=False`` renders with brute-force
    scans (RT_CFG_CULL = 0: every object tested by every ray; same bits, many times slower)."""

    def __init__(self, scene, width: int, height: int, depth: int, *, rank: int = 0, world: int = 1,
                 device: int = 0, row_block: int = 16, precision: str = "f32", order: str = "exact", group=None,
                 levels: bool = False, spp: int = 1, seed: int = 0, inflight: int = 1, cull: bool = True,
                 priorities="auto", assemble: bool = False):
        import torch
        self.torch = torch
        self.L = N.lib()
        self.w, self.h, self.depth = width, height, depth
        self.rank, self.world, self.rb, self.group = rank, world, row_block, group
        # assemble (world > 1): rank 0 renders no rows and only reassembles the frame; ranks 1 ..
        # world-1 render shards 0 .. world-2.  Rank 0 keeps contexts of shard 0's geometry for
        # launch_on (timing) only: launch() renders nothing there.
        self.assemble = bool(assemble) and world > 1
        self.nshards = world - 1 if self.assemble else world
        self.shard = max(rank - 1, 0) if self.assemble else rank
        self.renders = not (self.assemble and rank == 0)
        self.spp, self.seed = spp, seed
        self.prec, self.order = PRECISIONS[precision], ORDERS[order]
        self.precision = precision
        self.dtype = torch.float64 if precision == "f64" else torch.float32
        self.device = torch.device("cuda", device)
        self.rows = shard_rows(height, row_block, self.nshards)
        if inflight < 1 or (inflight > 1 and levels):
            raise ValueError("inflight must be >= 1 (and 1 with levels)")
        el = N.marshal(scene)
        self._ps = []
        for _ in range(inflight):
            p = ctypes.c_void_p()
            N.check(self.L.rt_prepare(el, len(el), device, ctypes.byref(p)), "rt_prepare")
            self._ps.append(p)
            if inflight > 1:
                N.check(self.L.rt_configure(p, N.RT_CFG_SIDE_STREAMS, 0), "rt_configure")
            if not cull:  # brute-force scans (RT_CFG_CULL = 0): the filters' bit-for-bit check
                N.check(self.L.rt_configure(p, N.RT_CFG_CULL, 0), "rt_configure")
        self._p = self._ps[0]
        self.slabs = [torch.empty((self.rows, width, 3), dtype=self.dtype, device=self.device)
                      for _ in range(inflight)]
        self.slab = self.slabs[0]
        # priorities (inflight > 1): one torch stream priority per slot (lower = higher priority; HIP
        # has two levels, 0 and -1).  "auto": with 4 or more frames in flight and one sample per pixel
        # the first half of the slots run at high priority.  Frames in flight on equal-priority
        # streams start in lockstep and stay there — their latency-bound tails (sparse deep levels,
        # the chain walk) coincide; the two classes keep the frames staggered, so one pair's dense
        # kernels fill the other pair's tails.  Measured, S64 4096^2 d5 (profiles/r05h_ab_priorities.txt):
        # 20 frames 0.436 -> 0.423 ms per frame, 100 frames 0.425 -> 0.412; S256 d8 x16 spp -0.7 %, so
        # not for supersampled frames.
        if priorities == "auto":
            priorities = [-1] * (inflight // 2) + [0] * (inflight - inflight // 2) \
                if inflight >= 4 and spp == 1 else None
        pr = list(priorities) if priorities is not None else [0] * inflight
        if not pr or len(pr) > inflight or any(p not in (0, -1) for p in pr):
            raise ValueError(f"priorities: 1 to {inflight} values, each 0 or -1 (HIP's two stream priorities), "
                             f"got {pr!r}; a shorter list is repeated over the frames in flight")
        self.streams = [torch.cuda.Stream(self.device, priority=pr[i % len(pr)]) for i in range(inflight)] \
            if inflight > 1 else None
        self.stream = torch.cuda.current_stream(self.device)
        self.n = 0
        self.levels = torch.empty((self.rows, width), dtype=torch.uint8, device=self.device) if levels else None
        self.gather_buf = None
        self.frame = None
        if world > 1 and rank == 0:
            if not self.assemble:  # (the dense gather's buffer; the compact gather has its own)
                self.gather_buf = torch.empty((world, self.rows, width, 3), dtype=self.dtype, device=self.device)
            self.frame = torch.empty((height, width, 3), dtype=self.dtype, device=self.device)
        self._pipe = None
        self._cg = None

    def launch(self):
        """Render the next frame: on the caller's current stream, or (inflight > 1) on the
        next slot's stream into that slot's slab."""
        j = self.n % len(self._ps)
        self.n += 1
        if self.streams is not None:
            self.slab, self.stream = self.slabs[j], self.streams[j]
        else:
            self.stream = self.torch.cuda.current_stream(self.device)
        if not self.renders:  # an assembling rank 0
            return
        lv = self.levels.data_ptr() if self.levels is not None else None
        N.check(self.L.rt_launch_spp(self._ps[j], self.w, self.h, self.depth, self.rb, self.shard, self.nshards,
                                     self.prec, self.order, self.spp, self.seed, self.slab.data_ptr(), lv,
                                     self.stream.cuda_stream), "rt_launch")

    def launch_on(self, j: int):
        """Render a frame on slot j's context, slab and stream (no gather)."""
        stream = self.streams[j] if self.streams is not None else self.torch.cuda.current_stream(self.device)
        N.check(self.L.rt_launch_spp(self._ps[j], self.w, self.h, self.depth, self.rb, self.shard, self.nshards,
                                     self.prec, self.order, self.spp, self.seed, self.slabs[j].data_ptr(), None,
                                     stream.cuda_stream), "rt_launch")

    def time_kernels(self, mask: int):
        """Bracket every later launch of the RT_KT_* kernels in `mask` with HIP events on the
        stream each runs on (every slot context); 0 stops."""
        for p in self._ps:
            N.check(self.L.rt_configure(p, N.RT_CFG_KERNEL_TIMING, mask), "rt_configure")
            for k in (N.RT_KT_PRIMARY, N.RT_KT_LEVEL1, N.RT_KT_RENDER, N.RT_KT_PMASK):
                N.check(self.L.rt_kernel_time(p, k, None, None, 1), "rt_kernel_time")  # reset

    def kernel_time(self, kernel: int):
        """(average ms per launch, launches) of an RT_KT_* kernel over every slot context since
        time_kernels(); waits for the recorded events."""
        tot, n = 0.0, 0
        for p in self._ps:
            ms, c = ctypes.c_double(0), ctypes.c_uint64(0)
            N.check(self.L.rt_kernel_time(p, kernel, ctypes.byref(ms), ctypes.byref(c), 0), "rt_kernel_time")
            tot += ms.value
            n += c.value
        return (tot / n if n else None), n

    def fork(self):
        """Make every slot stream wait for the caller's current stream (start of a timed region)."""
        if self.streams is not None:
            cur = self.torch.cuda.current_stream(self.device)
            for s in self.streams:
                s.wait_stream(cur)

    def join(self):
        """Make the caller's current stream wait for every slot stream."""
        if self.streams is not None:
            cur = self.torch.cuda.current_stream(self.device)
            for s in self.streams:
                cur.wait_stream(s)

    def gather(self):
        if self.world == 1:
            return self.slab
        if self.assemble:
            raise ValueError("an assembling rank 0 takes the compact gather (compact_gather)")
        import torch.distributed as dist
        if self.rank == 0:
            dist.gather(self.slab, gather_list=list(self.gather_buf.unbind(0)), dst=0, group=self.group)
            st = self.torch.cuda.current_stream(self.device).cuda_stream
            N.check(self.L.rt_unshard(self.gather_buf.data_ptr(), self.w, self.h, self.rb, self.world, self.prec,
                                      self.frame.data_ptr(), st), "rt_unshard")
            return self.frame
        dist.gather(self.slab, gather_list=None, dst=0, group=self.group)
        return None

    def step(self):
        self.launch()
        return self.gather()

    # ---- pipelined frames (world > 1): render frame i+1 while frame i is gathered ----------
    def pipeline(self):
        if self.assemble:
            raise ValueError("an assembling rank 0 takes the compact gather (compact_gather)")
        if self.streams is not None:
            raise ValueError("the dense slab pipeline takes one frame in flight (inflight=1)")
        if self._pipe is None:
            torch = self.torch
            slabs = [self.slab, torch.empty_like(self.slab)]
            gbufs = [self.gather_buf, torch.empty_like(self.gather_buf)] if self.gather_buf is not None else None
            self._pipe = SlabPipeline(self.world, self.rank, slabs, gbufs, self._reorder, self.group)
        return self._pipe

    def _reorder(self, gbuf):
        st = self.torch.cuda.current_stream(self.device).cuda_stream
        N.check(self.L.rt_unshard(gbuf.data_ptr(), self.w, self.h, self.rb, self.world, self.prec,
                                  self.frame.data_ptr(), st), "rt_unshard")
        return self.frame

    def step_pipelined(self):
        """Render the next frame into the free slab and start its gather; returns the previous
        frame on rank 0 once its gather has completed (None otherwise).  drain() finishes."""
        pipe = self.pipeline()
        self.slab = pipe.slab
        self.launch()
        return pipe.submit()

    def drain(self):
        return self._pipe.drain() if self._pipe is not None else None

    # ---- compact gather (world > 1, the default in bench.py): background pixels not sent ----
    def compact_gather(self):
        if self._cg is None:
            codec = SlabCodec(self.w, self.h, self.rb, self.nshards, self.precision)
            self._cg = CompactGather(codec, self.world, self.rank, self.slab.numel(), self.dtype, self.device,
                                     self.frame, self.group, first=1 if self.assemble else 0)
        return self._cg

    def step_compact(self):
        """Render the next frame and hand it to the compact gather; returns (rank 0) the frame
        two steps back once decoded, None otherwise.  drain_compact() finishes."""
        cg = self.compact_gather()
        self.launch()
        with self.torch.cuda.stream(self.stream):
            return cg.submit(self.slab if self.renders else None, self.shard)

    def drain_compact(self):
        return self._cg.drain() if self._cg is not None else None

    def close(self):
        for p in self._ps:
            if p:
                self.L.rt_release(p)
        self._ps = []
        self._p = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
