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


class FrameRenderer:
    """Renders this rank's rows of a W x H frame on its GPU and gathers the frame to rank 0.

    ``step()`` = one pass of the hot path over one frame: the render kernel on this
    rank's rows (rt_launch) and, for world > 1, the gather plus rank 0's reorder
    (rt_unshard, two strided device copies)."""

    def __init__(self, scene, width: int, height: int, depth: int, *, rank: int = 0, world: int = 1,
                 device: int = 0, row_block: int = 16, precision: str = "f32", order: str = "exact", group=None,
                 levels: bool = False, spp: int = 1, seed: int = 0):
        import torch
        self.torch = torch
        self.L = N.lib()
        self.w, self.h, self.depth = width, height, depth
        self.rank, self.world, self.rb, self.group = rank, world, row_block, group
        self.spp, self.seed = spp, seed
        self.prec, self.order = PRECISIONS[precision], ORDERS[order]
        self.dtype = torch.float64 if precision == "f64" else torch.float32
        self.device = torch.device("cuda", device)
        self.rows = shard_rows(height, row_block, world)
        el = N.marshal(scene)
        self._p = ctypes.c_void_p()
        N.check(self.L.rt_prepare(el, len(el), device, ctypes.byref(self._p)), "rt_prepare")
        self.slab = torch.empty((self.rows, width, 3), dtype=self.dtype, device=self.device)
        self.levels = torch.empty((self.rows, width), dtype=torch.uint8, device=self.device) if levels else None
        self.gather_buf = None
        self.frame = None
        if world > 1 and rank == 0:
            self.gather_buf = torch.empty((world, self.rows, width, 3), dtype=self.dtype, device=self.device)
            self.frame = torch.empty((height, width, 3), dtype=self.dtype, device=self.device)
        self._pipe = None

    def launch(self):
        st = self.torch.cuda.current_stream(self.device).cuda_stream
        lv = self.levels.data_ptr() if self.levels is not None else None
        N.check(self.L.rt_launch_spp(self._p, self.w, self.h, self.depth, self.rb, self.rank, self.world, self.prec,
                                     self.order, self.spp, self.seed, self.slab.data_ptr(), lv, st), "rt_launch")

    def gather(self):
        if self.world == 1:
            return self.slab
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

    def close(self):
        if self._p:
            self.L.rt_release(self._p)
            self._p = ctypes.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
