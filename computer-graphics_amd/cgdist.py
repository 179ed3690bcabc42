"""Multi-GPU raytracer sharding: framebuffer stripes dealt
round-robin over ranks, one gather to rank 0, one unstripe kernel.

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
