"""Multi-GPU raytracer sharding.  The product path is native:
cg_rt_render_frames_dist (csrc/cg_dist.hip: balanced bands, RCCL p2p to rank
0, in-place assembly); join() below sets it up over a torch.distributed
world.  This module also keeps the earlier stripe layout (framebuffer
stripes dealt round-robin over ranks, one gather to rank 0, one unstripe
kernel) and numpy mirrors of the partition / assembly logic for CPU tests.

Pixels are independent in the reference's Draw (raytracer/Source/
skeleton.cpp:123-168), so there is no data-path exchange while rendering:
each rank renders `stripe_h`-row stripes k with k % nranks == rank (packed in
order, padded to the same row count on every rank so the gather moves
equal-size buffers), rank 0 gathers them over RCCL and reassembles the frame
on the device (cg_rt_unstripe_device).  Interleaved stripes balance the
row-dependent cost (sphere, shadows) far better than contiguous bands.

The numpy helpers mirror the device kernels' index maps for CPU tests.
"""
from __future__ import annotations

import numpy as np

DEFAULT_STRIPE = 8   # = the general RT kernel's tile height (cg_internal.h kRtTileH)
LATTICE_STRIPE = 15  # = the lattice kernel's tile height (cg_rt.hip kLatTileH): C2's stripes


def shard_rows(height: int, nranks: int, stripe_h: int = DEFAULT_STRIPE) -> int:
    """Rows each rank renders (cg_rt_shard_rows)."""
    stripes = -(-height // stripe_h)
    per = -(-stripes // nranks)
    return per * stripe_h


def shard_row_map(height: int, rank: int, nranks: int, stripe_h: int = DEFAULT_STRIPE) -> np.ndarray:
    """Global row of each local row of a rank's shard (>= height: padding)."""
    L = np.arange(shard_rows(height, nranks, stripe_h))
    k = L // stripe_h
    return (k * nranks + rank) * stripe_h + (L - k * stripe_h)


def unstripe_np(gathered: np.ndarray, height: int, nranks: int, stripe_h: int = DEFAULT_STRIPE) -> np.ndarray:
    """gathered: [nranks, rows, W] -> frame [height, W] (mirror of rt_unstripe_kernel)."""
    y = np.arange(height)
    k = y // stripe_h
    r = k % nranks
    L = (k // nranks) * stripe_h + (y - k * stripe_h)
    return gathered[r, L]


# ---- balanced bands (the default multi-GPU layout) -------------------------
# Each rank renders one contiguous band of rows, so rank 0 can receive every
# band straight into its row range: no unstripe pass, one p2p transfer per
# rank per batch of frames.  Band boundaries are chosen to equalise each
# rank's measured time (rank 0 also pays the frame assembly), re-estimated
# from per-rank timings during warm-up (rebalance()).

def equal_bands(height: int, nranks: int, align: int = 1):
    """Contiguous bands of (near) equal height, boundaries on multiples of `align`."""
    units = -(-height // align)
    bounds = [min(height, (units * r // nranks) * align) for r in range(nranks + 1)]
    bounds[-1] = height
    return [(bounds[r], bounds[r + 1] - bounds[r]) for r in range(nranks)]


def band_partition(row_cost, nranks: int, overhead=None):
    """Contiguous bands minimising max_r (sum of row_cost over band r + overhead[r]).
    Bisection on the makespan with a greedy sweep; every rank gets >= 1 row when
    there are enough rows.  Returns [(row0, rows)] in rank order."""
    c = np.asarray(row_cost, dtype=np.float64)
    H = len(c)
    o = np.zeros(nranks) if overhead is None else np.asarray(overhead, dtype=np.float64)
    C = np.concatenate([[0.0], np.cumsum(c)])

    def sweep(T):
        b = [0]
        for r in range(nranks - 1):
            lo = b[-1]
            left = nranks - 1 - r                    # ranks still to place after this one
            hi_max = max(lo + 1, H - left) if H >= nranks else lo + (1 if lo < H else 0)
            # largest end with cost <= T (at least one row, leaving one per later rank)
            end = int(np.searchsorted(C, C[lo] + T - o[r], side="right")) - 1
            end = min(max(end, lo + 1 if lo < H else lo), hi_max)
            b.append(end)
        b.append(H)
        return b

    lo_T, hi_T = 0.0, C[-1] + o.max() + 1.0
    for _ in range(60):
        T = 0.5 * (lo_T + hi_T)
        b = sweep(T)
        last = C[b[-1]] - C[b[-2]] + o[nranks - 1]
        if last <= T:
            hi_T = T
        else:
            lo_T = T
    b = sweep(hi_T)
    return [(b[r], b[r + 1] - b[r]) for r in range(nranks)]


def rebalance(bands, render_s, overhead_s, height: int):
    """New bands from measured per-rank render times (cost density uniform within
    each old band) and per-rank fixed overheads (rank 0's assembly)."""
    cost = np.zeros(height)
    for (r0, n), t in zip(bands, render_s):
        if n > 0:
            cost[r0:r0 + n] = max(float(t), 1e-12) / n
    return band_partition(cost, len(bands), overhead_s)


def join(ctx, group=None, chunk=None, timeout_ms=0):
    """This process's cgamd.Dist in the torch.distributed world (one process
    per GPU): rank 0 creates the RCCL id (cg_dist_unique_id) and it travels
    over the existing process group; cg_dist_create_timed then joins the
    library's own RCCL communicator on ctx's device (non-blocking, every host
    wait bounded by timeout_ms; 0 = the library's default)."""
    import torch
    import torch.distributed as dist

    import cgamd
    rank, world = dist.get_rank(group), dist.get_world_size(group)
    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend(group) == "nccl" else "cpu"
    t = torch.zeros(cgamd.DIST_ID_BYTES, dtype=torch.uint8, device=dev)
    if rank == 0:
        t.copy_(torch.tensor(list(cgamd.dist_unique_id()), dtype=torch.uint8))
    dist.broadcast(t, src=0, group=group)
    d = cgamd.Dist(ctx, world, rank, bytes(t.cpu().tolist()), timeout_ms=timeout_ms)
    if chunk:
        d.set_chunk(chunk)
    return d


def pack_rgb24_np(argb: np.ndarray) -> np.ndarray:
    """CG_PIX_RGB24 of ARGB8888 pixels: the low three bytes (B, G, R) of each."""
    return argb.astype("<u4").view(np.uint8).reshape(-1, 4)[:, :3].reshape(-1).copy()


def window_np(rows_px: np.ndarray, width: int, col0: int, cols: int) -> np.ndarray:
    """The window columns col0 .. col0 + cols - 1 of rows of `width` pixels (flattened)."""
    return rows_px.reshape(-1, width)[:, col0:col0 + cols].reshape(-1)


def assemble_np(src: np.ndarray, bpp: int, bands, width: int, height: int, nframes: int, frames: np.ndarray,
                col0: int = 0, cols: int = 0):
    """Mirror of rt_assemble_kernel: src = blocks in order, block b = nframes x
    rows_b rows (of the window's `cols` pixels when cols > 0, the rest black);
    frames [nframes, height*width] uint32 updated in place."""
    pitch = cols if cols else width
    c0 = col0 if cols else 0
    off = 0
    for r0, n in bands:
        for f in range(nframes):
            blk = src[off:off + n * pitch * bpp]
            off += n * pitch * bpp
            if bpp == 4:
                px = blk.view("<u4")
            else:
                b3 = blk.reshape(-1, 3).astype(np.uint32)
                px = 0x80000000 | b3[:, 0] | (b3[:, 1] << 8) | (b3[:, 2] << 16)
            rows = min(n, max(0, height - r0))
            full = np.full((rows, width), 0x80000000, np.uint32)
            full[:, c0:c0 + pitch] = px[:rows * pitch].reshape(rows, pitch)
            frames[f, r0 * width:(r0 + rows) * width] = full.reshape(-1)
    return frames
