"""Test-side restatement of the compact slab format (include/rt_mi355x.h, "compact slab
transfer"; the HIP codec is eraytracer_amd/csrc/rt_slab.hip).  Torch CPU ops, used as the
checker of the HIP codec on the GPU and as a stand-in codec for the gloo tests of
eraytracer_amd.dist.CompactGather.  Not part of the product.

Header of one shard's slab (rows = rt_shard_rows(H, rb, ns), px = rows * W):
    bytes [0, 8)          u64 count of non-zero pixels
    bytes [64, 64+4*nblk) u32 per 256-pixel block: non-zero pixels before it
    bytes [mask_at, ...)  u64 per 64 pixels: bit j = pixel 64*w + j is non-zero
with nblk = ceil(px/256), mask_at = roundup(64 + 4*nblk, 256), size = mask_at + 32*nblk.
A pixel is non-zero iff any of its three channels has a non-zero bit pattern; slab rows past
the image count as zero.  Values: the non-zero pixels' three channels in slab order.
"""
import numpy as np
import torch

from eraytracer_amd.dist import shard_global_rows, shard_rows


def layout(width, height, row_block, nshards):
    px = shard_rows(height, row_block, nshards) * width
    nblk = -(-px // 256)
    mask_at = (64 + 4 * nblk + 255) // 256 * 256
    return px, nblk, mask_at, mask_at + 32 * nblk


def _bits(t):
    return t.view({4: torch.int32, 8: torch.int64}[t.element_size()])


def nonzero_mask(slab, width, height, row_block, nshards, shard):
    rows = shard_rows(height, row_block, nshards)
    valid = torch.from_numpy(shard_global_rows(height, row_block, nshards, shard) >= 0)
    nz = (_bits(slab.reshape(rows, width, 3)) != 0).any(-1) & valid[:, None]
    return nz.reshape(-1)


class RefCodec:
    def __init__(self, width, height, row_block, world):
        self.w, self.h, self.rb, self.world = width, height, row_block, world
        self.px, self.nblk, self.mask_at, self.header_bytes = layout(width, height, row_block, world)

    def pack(self, slab, shard, header, values):
        nz = nonzero_mask(slab, self.w, self.h, self.rb, self.world, shard)
        pad = torch.zeros(self.nblk * 256, dtype=torch.bool)
        pad[: self.px] = nz
        words = pad.reshape(-1, 64).to(torch.int64) << torch.arange(64, dtype=torch.int64)
        mask = words.sum(1)  # wraps into the sign bit for bit 63, as u64 bits
        per_blk = pad.reshape(-1, 256).sum(1).to(torch.int64)
        off = torch.cumsum(per_blk, 0) - per_blk
        header.zero_()
        header[:8] = torch.tensor([int(nz.sum())], dtype=torch.int64).view(torch.uint8)
        header[64: 64 + 4 * self.nblk] = off.to(torch.int32).view(torch.uint8)
        header[self.mask_at:] = mask.view(torch.uint8)
        flat = slab.reshape(-1, 3)[: self.px]
        sel = flat[nz]
        values[: sel.numel()] = sel.reshape(-1)

    def unpack(self, headers, values, frame):
        out = frame.reshape(self.h, self.w, 3)
        out.zero_()
        rows = shard_rows(self.h, self.rb, self.world)
        for s in range(self.world):
            hdr = headers[s]
            words = hdr[self.mask_at:].view(torch.int64)
            bits = ((words[:, None] >> torch.arange(64, dtype=torch.int64)) & 1).reshape(-1)[: self.px].bool()
            n = int(hdr[:8].view(torch.int64)[0])
            assert int(bits.sum()) == n
            slab = torch.zeros((self.px, 3), dtype=frame.dtype)
            slab[bits] = values[s][: 3 * n].reshape(n, 3)
            g = shard_global_rows(self.h, self.rb, self.world, s)
            keep = np.nonzero(g >= 0)[0]
            out[torch.from_numpy(g[keep])] = slab.reshape(rows, self.w, 3)[torch.from_numpy(keep)]
