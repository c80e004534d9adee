"""Film partitioning across ranks.

Stripes of ``stripe_height`` rows go round-robin to ranks (stripe k -> rank
k mod N). A rank renders the 8-row pixel bands (the 8x8 wave block height)
that touch its stripes or their ``halo`` rows, and convolves only the rows it
owns, so the sum of all ranks' films equals the one-GPU film bit for bit.
This mirrors ``dcrt_tracer::BuildBands`` / ``film_kernel`` in csrc/device.
"""
from __future__ import annotations

import numpy as np

BLOCK_H = 8
DEFAULT_HALO = 2


def owned_rows(height: int, world_size: int, rank: int, stripe_height: int) -> np.ndarray:
    y = np.arange(height)
    if world_size <= 1:
        return np.ones(height, bool)
    return (y // stripe_height) % world_size == rank


def render_bands(height: int, world_size: int, rank: int, stripe_height: int, halo: int = DEFAULT_HALO) -> list:
    """First rows of the 8-row bands this rank path-traces."""
    if world_size <= 1:
        return list(range(0, height, BLOCK_H))
    own = owned_rows(height, world_size, rank, stripe_height)
    need = np.zeros(height, bool)
    for y in np.nonzero(own)[0]:
        need[max(0, y - halo):min(height - 1, y + halo) + 1] = True
    return [y for y in range(0, height, BLOCK_H) if need[y:y + BLOCK_H].any()]


def owned_row_ranges(height: int, world_size: int, rank: int, stripe_height: int) -> list:
    own = owned_rows(height, world_size, rank, stripe_height)
    out, y = [], 0
    while y < height:
        if own[y]:
            y1 = y
            while y1 < height and own[y1]:
                y1 += 1
            out.append((y, y1))
            y = y1
        else:
            y += 1
    return out
