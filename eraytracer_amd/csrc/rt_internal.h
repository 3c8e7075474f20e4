// rt_internal.h — entry points shared between the library's translation units (not part of
// the C ABI in include/rt_mi355x.h).
#pragma once
#include <hip/hip_runtime.h>

#include <stddef.h>
#include <stdint.h>

#include "../../include/rt_mi355x.h"

// rt_launch_spp restricted to slab rows [row_begin, min(row_end, slab rows)) (rt_render.hip).
// row_begin must be a multiple of 16 (the tile height); d_out / d_levels point at slab row 0.
// levels_hit: d_levels gets the primary-hit mask (1 / 0) instead of the level count (RT_LEVELS_HIT).
int rt_launch_rows(rt_prepared *p, uint32_t width, uint32_t height, uint32_t depth, uint32_t row_block,
                   uint32_t shard, uint32_t nshards, int precision, int order, uint32_t spp, uint64_t seed,
                   uint32_t row_begin, uint32_t row_end, void *d_out, uint8_t *d_levels, void *stream,
                   int levels_hit = 0);

// Replace the scene of a prepared context in place (its work space, streams and events are
// kept; captured frame graphs are invalidated).  No launch of p may be in flight.
int rt_prepare_scene(rt_prepared *p, const rt_elem *scene, uint32_t n);

// Free p's wavefront work space (queues, colours, flags, lists, supersampling sums, primary
// masks: GBs at 4096^2); the next launch grows it again.  No launch of p may be in flight.
// Returns the bytes freed.
size_t rt_trim(rt_prepared *p);

// ---- the process's render contexts (rt_host.hip) ------------------------------------------
// One context = one device, two streams (render, copy), the most recently prepared scene with
// its grown work space, grown device output buffers and a pinned host staging buffer.  The
// pool keeps them across calls (one lazily initialised context per process;
// up to RT_CTX_PER_DEVICE concurrent callers per device get one each).
struct rt_ctx;
// Take a free context of `device` with `scene` prepared on it (compiled and uploaded only when
// it differs from the context's last scene).  Blocks while every context of the device is busy.
int rt_ctx_acquire(int device, const rt_elem *scene, uint32_t n, rt_ctx **out);
void rt_ctx_release(rt_ctx *c);
rt_prepared *rt_ctx_prepared(rt_ctx *c);
hipStream_t rt_ctx_stream(rt_ctx *c);
// Device buffer `which` (0..2) of at least `bytes`, kept (and grown) with the context.
int rt_ctx_device_buffer(rt_ctx *c, int which, size_t bytes, void **out);
// Pinned host staging buffer of at least `bytes`, kept with the context.
int rt_ctx_host_buffer(rt_ctx *c, size_t bytes, void **out);
