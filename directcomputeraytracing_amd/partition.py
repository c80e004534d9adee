"""Film partitioning across ranks.

The H film rows are cut into K = N * k stripes of floor/ceil(H / K) rows, with
k = round(H / (N * stripe_height)) (at least 1): stripe j covers rows
[j*H/K, (j+1)*H/K) and belongs to rank j mod N, so every rank owns k stripes and
the same number of rows to within one per stripe. A rank path-traces its rows
plus ``halo`` rows beyond each stripe edge (the filter's support, floor(r + 0.5)
rows) and convolves only the rows it owns, so the sum of all ranks' films equals
the one-GPU film bit for bit. The rendered rows are packed 8 per block row in
ascending order. This mirrors ``dcrt_tracer::BuildRows`` / ``film_kernel`` in
csrc/device.
"""
from __future__ import annotations

import numpy as np

BLOCK_H = 8
DEFAULT_HALO = 2


def stripe_count(height: int, world_size: int, stripe_height: int) -> int:
    k = max(1, (height + (world_size * stripe_height) // 2) // (world_size * stripe_height))
    return min(world_size * k, height)


def owned_rows(height: int, world_size: int, rank: int, stripe_height: int) -> np.ndarray:
    if world_size <= 1:
        return np.ones(height, bool)
    K = stripe_count(height, world_size, stripe_height)
    own = np.zeros(height, bool)
    for j in range(rank, K, world_size):
        own[j * height // K:(j + 1) * height // K] = True
    return own


def render_rows(height: int, world_size: int, rank: int, stripe_height: int, halo: int = DEFAULT_HALO) -> list:
    """Rows this rank path-traces, ascending (8 of them per block row)."""
    if world_size <= 1:
        return list(range(height))
    K = stripe_count(height, world_size, stripe_height)
    need = np.zeros(height, bool)
    for j in range(rank, K, world_size):
        y0, y1 = j * height // K, (j + 1) * height // K
        need[max(0, y0 - halo):min(height, y1 + halo)] = True
    return [int(y) for y in np.nonzero(need)[0]]


def stream_partition(height: int, world_size: int, rank: int, streams: int, stream: int, stripe_height: int):
    """(world, rank, stripe height) of pipeline `stream` of the `streams` concurrent ones on
    rank `rank` of `world_size`: virtual rank s * N + r of N * K. Any such split is exact
    (the virtual ranks' films have disjoint supports); the stripe height is chosen so the
    N * K virtual ranks share about as many stripes as the N ranks do without streams
    (then, when K divides them, a rank owns exactly its stripes of the K = 1 split, dealt
    round-robin to its pipelines and no halo row is added). One GPU: K horizontal bands."""
    if world_size <= 1:
        return streams, stream, -(-height // streams)
    total = stripe_count(height, world_size, stripe_height)
    v = world_size * streams
    k = max(1, round(total / v))
    return v, stream * world_size + rank, max(1, round(height / (v * k)))


def band_render_rows(height: int, bands, halo: int = DEFAULT_HALO) -> list:
    """Rows a tracer with explicit film bands path-traces (dcrt_tracer::BuildRows): its bands'
    rows plus `halo` rows beyond each, ascending."""
    need = np.zeros(height, bool)
    for y0, y1 in bands:
        y0, y1 = min(y0, height), min(y1, height)
        if y0 < y1:
            need[max(0, y0 - halo):min(height, y1 + halo)] = True
    return [int(y) for y in np.nonzero(need)[0]]


def band_owned_rows(height: int, bands) -> np.ndarray:
    own = np.zeros(height, bool)
    for y0, y1 in bands:
        own[min(y0, height):min(y1, height)] = True
    return own


def band_cost(prefix: np.ndarray, y0: int, y1: int, halo: int) -> float:
    """Cost of path-tracing band [y0, y1) with its halo rows: the rows' summed cost."""
    h = len(prefix) - 1
    return float(prefix[min(h, y1 + halo)] - prefix[max(0, y0 - halo)])


def balanced_bands(row_cost, parts: int, halo: int = DEFAULT_HALO) -> list:
    """Cut the film's rows into `parts` contiguous bands [y0, y1) whose largest cost -- the
    summed per-row cost of the band and of the halo rows its tracer also path-traces -- is as
    small as contiguous cuts allow (balance scene-dependent cost). Row costs come
    from the tracer's row-cost probe (rays per row, tracer.probe_row_cost). Deterministic: ranks
    that probe the same scene get the same cuts. Returns `parts` bands covering every row once."""
    c = np.maximum(np.asarray(row_cost, np.float64), 0.0)
    H = len(c)
    parts = max(1, min(int(parts), H))
    if parts == 1:
        return [(0, H)]
    c = c + 1e-9 * max(1.0, c.max())   # (every row costs something: empty rows still take slots)
    P = np.concatenate([[0.0], np.cumsum(c)])

    def greedy(T):
        """Bands of cost <= T taken greedily from the top (each at least one row); None if more
        than `parts` are needed."""
        cuts, y0 = [], 0
        while y0 < H:
            if len(cuts) == parts:
                return None
            y1 = y0 + 1
            lo, hi = y0 + 1, H   # the largest y1 with cost <= T (cost grows with y1)
            while lo <= hi:
                mid = (lo + hi) // 2
                if band_cost(P, y0, mid, halo) <= T:
                    y1, lo = mid, mid + 1
                else:
                    hi = mid - 1
            cuts.append((y0, y1))
            y0 = y1
        return cuts

    lo = max(band_cost(P, y, y + 1, halo) for y in range(H))
    hi = band_cost(P, 0, H, halo)
    best = greedy(hi)
    for _ in range(64):   # bisection on the bottleneck cost
        mid = 0.5 * (lo + hi)
        g = greedy(mid)
        if g is None:
            lo = mid
        else:
            hi, best = mid, g
        if hi - lo <= 1e-6 * hi:
            break
    bands = list(best)
    # fewer bands than parts: split the costliest band in two (a sub-band costs no more)
    while len(bands) < parts:
        i = max((k for k in range(len(bands)) if bands[k][1] - bands[k][0] > 1),
                key=lambda k: band_cost(P, bands[k][0], bands[k][1], halo))
        y0, y1 = bands[i]
        # the split row that balances the two halves
        m = min(range(y0 + 1, y1), key=lambda y: max(band_cost(P, y0, y, halo), band_cost(P, y, y1, halo)))
        bands[i:i + 1] = [(y0, m), (m, y1)]
    return [(int(a), int(b)) for a, b in bands]


def refine_row_cost(row_cost, rank_bands, rank_times, halo: int = DEFAULT_HALO) -> np.ndarray:
    """Row costs corrected by measured time: rank r rendered rank_bands[r] (with halo) in
    rank_times[r]; every row it owns is rescaled by r's time per unit of modelled cost. The
    probe's rays are not time (time per ray grows down the Cornell image: more node visits and
    triangle tests per ray), so one calibration run of the cut bands, gathered from all ranks,
    re-cuts them at equal time. Deterministic given the gathered times: every rank computes the
    same vector."""
    c = np.maximum(np.asarray(row_cost, np.float64), 0.0)
    P = np.concatenate([[0.0], np.cumsum(c)])
    out = c.copy()
    for bands, t in zip(rank_bands, rank_times):
        modelled = sum(band_cost(P, y0, y1, halo) for y0, y1 in bands)
        if modelled <= 0 or not t > 0:
            continue
        for y0, y1 in bands:
            out[y0:y1] = c[y0:y1] * (float(t) / modelled)
    return out * (P[-1] / max(out.sum(), 1e-300))   # (the same total as the input)


def pipeline_pool(pool: int, rows: int, width: int, images: int, max_batch: int = 256, slack: float = 0.08) -> int:
    """Path-pool slots for one pipeline rendering `images` images of `rows` x `width` pixels.

    dcrt_tracer::AutoBatch cuts a render into equal batches of as many images as the pool
    holds (at most `max_batch`), and every batch ends in a drain. When the pool falls just
    short of a whole number of batches (an N = 8 rank's stripes plus halo: 62.4 shares of a
    2^23 pool, i.e. 5 batches of 256 shares instead of 4) the pool grows by up to `slack`
    so the render needs one batch less; otherwise it is returned unchanged. An image takes
    whole 8x8 pixel blocks of slots (partial bands and columns included), as AutoBatch counts."""
    px = max(1, -(-rows // BLOCK_H) * BLOCK_H * -(-width // 8) * 8)
    batches = max(-(-images // max_batch), -(-int(images * px) // int(pool * (1.0 + slack))))
    need = -(-images // batches) * px
    return max(pool, -(-need // 256) * 256)


def halo_for_radius(radius: float, height: int = 65535) -> int:
    """Rows of support beyond a pixel row that SampleConvolution gathers (SampleConvolution.hlsl:77-81),
    in the kernel's float32 arithmetic over the film's rows (dcrt_tracer FilterSupportRows): floor(r + 0.5),
    or one more where py + 0.5 + r rounds up to an integer (r just below k + 0.5)."""
    r = np.float32(radius)
    if not r < height:
        return int(height)
    py = np.arange(height, dtype=np.int64)
    cy = py.astype(np.float32) + np.float32(0.5)
    ys = np.maximum(np.floor(cy - r).astype(np.int64), 0)
    ye = np.minimum(np.floor(cy + r).astype(np.int64), height - 1)
    return int(max(int((ye - py).max()), int((py - ys).max()), 0))


def row_runs(rows) -> list:
    """Contiguous (y0, y1) runs of an ascending row list."""
    out = []
    for y in rows:
        if out and out[-1][1] == y:
            out[-1][1] = y + 1
        else:
            out.append([y, y + 1])
    return [tuple(r) for r in out]


def owned_row_ranges(height: int, world_size: int, rank: int, stripe_height: int) -> list:
    return row_runs(np.nonzero(owned_rows(height, world_size, rank, stripe_height))[0])
