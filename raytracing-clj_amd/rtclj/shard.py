"""Multi-GPU work split of one frame (the reference's row-chunk executor,
raytracing.clj:157-171, redesigned for N GPUs of one node).

Two decompositions, both collective-free (pixels are independent and the RNG
is keyed by (seed, pixel, sample), so every shard computes exactly what a
single device would for its pixels/samples):

  strong — one frame, interleaved row tiles: tile t (row_tile rows) goes to
           rank t % world.  Sky-only and ground/glass-heavy rows are spread
           over every rank (contiguous halves, as the reference's 2-thread
           pool uses, would leave the top-of-frame rank idle).
  weak   — every rank renders the whole frame with its own sample stripe
           [rank*spp, (rank+1)*spp); stripes average into a world*spp frame.

The host gather puts compacted tile rows back in image order.
"""
from __future__ import annotations

import numpy as np


def shard_rows(height, row_tile=8, tile_first=0, tile_step=0, row_begin=0, row_end=None):
    """Global rows a shard renders, in its compacted output order.

    Restates the kernel's output-row -> image-row map (trace.hip, "compacted
    output row -> global image row") and rt_rows_out."""
    row_end = height if row_end is None else row_end
    if tile_step <= 0:
        return list(range(row_begin, row_end))
    span = row_end - row_begin
    ntiles = -(-span // row_tile)
    rows = []
    for t in range(tile_first, ntiles, tile_step):
        rows.extend(range(row_begin + t * row_tile, row_begin + min(span, (t + 1) * row_tile)))
    return rows


def shard_params(world, rank, width, height, spp, max_depth, seed=1, scaling="strong", row_tile=8):
    """rt_params fields for `rank` of `world` (see module doc)."""
    if not 0 <= rank < world:
        raise ValueError(f"rank {rank} outside world {world}")
    base = dict(width=width, height=height, row_begin=0, row_end=height, spp=spp, max_depth=max_depth, seed=seed)
    if scaling == "weak":
        return dict(base, sample_begin=rank * spp)
    if scaling != "strong":
        raise ValueError(f"scaling {scaling!r}")
    if world == 1:
        return dict(base, row_tile=row_tile)
    return dict(base, row_tile=row_tile, tile_first=rank, tile_step=world)


def gather_rows(height, width, parts):
    """parts: [(rows, array (len(rows), width, 3))] -> full (height, width, 3) frame.

    Each image row must be covered exactly once."""
    out = np.zeros((height, width, 3), np.float32)
    seen = np.zeros(height, np.int32)
    for rows, arr in parts:
        arr = np.asarray(arr).reshape(len(rows), width, 3)
        out[rows] = arr
        seen[rows] += 1
    if not (seen == 1).all():
        raise ValueError(f"rows covered {seen.min()}..{seen.max()} times")
    return out
