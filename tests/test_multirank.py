"""Film partitioning across ranks on CPU with gloo, world size 2.

Each rank path-traces only the rows of its round-robin stripes plus a 1-row
halo (directcomputeraytracing_amd.partition, mirroring dcrt_tracer::BuildRows),
convolves only the rows it owns, and one reduce(SUM) of the RGBA32F film
yields the single-rank film bit for bit. The per-rank rendering here is the
oracle (no GPU in this container); the GPU path is covered by
test_gpu_parity.py::test_film_partition_sums_to_single_gpu.
"""
import os
import socket

import numpy as np
import pytest

from conftest import GOLDEN, ROOT


def test_halo_for_radius_matches_window_arithmetic():
    """halo_for_radius = the furthest row a window [floor(py + 0.5 - r), floor(py + 0.5 + r)] reaches,
    in float32 (film_kernel's arithmetic): floor(r + 0.5), one more for r just below k + 0.5."""
    from directcomputeraytracing_amd.partition import halo_for_radius
    below = lambda x: float(np.nextafter(np.float32(x), np.float32(0)))
    H = 1080
    for r in (0.5, 1.0, below(1.5), 1.5, 2.0, below(2.5), 2.5, 3.3, below(4.5)):
        r32 = np.float32(r)
        reach = 0
        for py in range(H):
            cy = np.float32(py) + np.float32(0.5)
            ys = max(0, int(np.floor(cy - r32)))
            ye = min(H - 1, int(np.floor(cy + r32)))
            reach = max(reach, ye - py, py - ys)
        assert halo_for_radius(r, H) == reach, r
    assert halo_for_radius(below(1.5), H) == 2 and halo_for_radius(1.0, H) == 1


def test_partition_rows_cover_film():
    from directcomputeraytracing_amd.partition import owned_rows, render_rows
    H, S = 1080, 64
    for world in (1, 2, 3, 4, 8):
        owners = np.stack([owned_rows(H, world, r, S) for r in range(world)])
        assert np.all(owners.sum(0) == 1)                      # every row owned exactly once
        counts = owners.sum(1)
        assert counts.max() - counts.min() <= max(1, H // (world * S))   # balanced to a row per stripe
        for halo in (1, 2):
            total = 0
            for r in range(world):
                rows = render_rows(H, world, r, S, halo)
                assert rows == sorted(set(rows))
                covered = np.zeros(H, bool)
                covered[rows] = True
                for y in np.nonzero(owners[r])[0]:             # owned rows +- halo rendered
                    assert covered[max(0, y - halo):min(H, y + halo + 1)].all()
                total += len(rows)
            if world > 1:
                assert total / H - 1 < 0.035 * halo            # halo overhead (16 stripes at S = 64)


def test_stream_partition_covers_film_once():
    """Concurrent pipelines per GPU (bench --streams K): virtual ranks s * N + r of N * K
    own every row exactly once, and with K = 2 a rank keeps exactly its K = 1 rows."""
    from directcomputeraytracing_amd.partition import owned_rows, stream_partition
    for H, S in ((1080, 64), (144, 16), (2160, 64), (97, 16)):
        for world in (1, 2, 3, 4, 8):
            for streams in (1, 2, 3):
                cover = np.zeros(H, int)
                for r in range(world):
                    mine = np.zeros(H, int)
                    for s in range(streams):
                        w, v, sh = stream_partition(H, world, r, streams, s, S)
                        assert 0 <= v < w == max(1, world * streams) or (world == 1 and w == streams)
                        mine += owned_rows(H, w, v, sh)
                    cover += mine
                    if world > 1 and streams == 2 and H == 1080:
                        assert np.array_equal(mine > 0, owned_rows(H, world, r, S))
                assert cover.min() == 1 and cover.max() == 1


def test_pipeline_pool_sizes_whole_batches():
    """bench.py's per-pipeline pool: unchanged at N = 1 (8 half-film shares fit 2^23
    slots), grown by at most 8 % where that saves a batch (N = 2 / 4 / 8 ranks' stripes
    plus halo at 8x8-block granularity), and the grown pool holds whole batches."""
    from directcomputeraytracing_amd.partition import pipeline_pool, render_rows, stream_partition
    W, H, base = 1920, 1080, 1 << 23

    def slots(rows):   # AutoBatch: whole 8x8 blocks
        return -(-rows // 8) * 8 * -(-W // 8) * 8

    for world in (1, 2, 4, 8):
        images = 64 * world
        for s in (0, 1):
            w, v, sh = stream_partition(H, world, 0, 2, s, 64)
            rows = len(render_rows(H, w, v, sh, 1))
            pool = pipeline_pool(base, rows, W, images)
            assert base <= pool <= base * 1.08 and pool % 256 == 0
            per = slots(rows)
            batch = min(64, pool // per)
            batches = -(-images // batch)
            assert batches <= -(-images // min(64, base // per))          # never more batches
            assert -(-images // batches) * per <= pool                     # equal batches fit
            if world == 1:
                assert pool == base
            if world == 8:
                assert batches == images // 64                             # 4 batches of 64, not 5


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_balanced_bands_cover_and_balance():
    """partition.balanced_bands: `parts` contiguous bands covering every row once, in order; the
    costliest band (with its halo rows) within one band-edge row of the best any contiguous cut
    can do (total / parts lower bound); deterministic; degenerate sizes handled."""
    from directcomputeraytracing_amd.partition import band_cost, band_owned_rows, band_render_rows, balanced_bands
    rng = np.random.default_rng(3)
    for H in (1, 7, 144, 1080, 2160):
        for parts in (1, 2, 3, 8, 16, 24):
            for halo in (1, 2):
                cost = rng.uniform(50, 400, H) * (1 + 3 * (np.arange(H) / max(1, H)) ** 2)
                bands = balanced_bands(cost, parts, halo)
                assert bands == balanced_bands(cost, parts, halo)
                assert len(bands) == min(parts, H) and bands[0][0] == 0 and bands[-1][1] == H
                assert all(a < b for a, b in bands) and all(bands[i][1] == bands[i + 1][0] for i in range(len(bands) - 1))
                P = np.concatenate([[0.0], np.cumsum(cost)])
                worst = max(band_cost(P, a, b, halo) for a, b in bands)
                bound = max(P[-1] / len(bands), max(band_cost(P, y, y + 1, halo) for y in range(H)))
                assert worst <= bound + (2 * halo + 1) * cost.max() + 1e-6
                own = sum(band_owned_rows(H, [b]).astype(int) for b in bands)
                assert (own == 1).all()
                for b in bands:
                    rows = band_render_rows(H, [b], halo)
                    assert rows[0] == max(0, b[0] - halo) and rows[-1] == min(H, b[1] + halo) - 1
    # a skewed cost moves the cuts: equal-cost bands are not equal-height bands
    cost = np.r_[np.full(500, 1.0), np.full(580, 10.0)]
    b = balanced_bands(cost, 2, 1)
    assert b[0][1] > 700


def _worker(rank, world, port, out_dir, mode="stripes"):
    import sys
    sys.path.insert(0, str(ROOT))
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import oracle
    from directcomputeraytracing_amd import FILTER_BOX, FilterParams, Scene, scenes
    from directcomputeraytracing_amd.partition import (balanced_bands, band_owned_rows, band_render_rows, owned_row_ranges,
                                                       render_rows, row_runs)
    W, H, S = 96, 80, 16
    if mode == "bands":
        # uneven contiguous bands, as the row-cost probe cuts them (a synthetic skewed cost here):
        # two per rank, like two pipelines of one GPU
        cost = 1.0 + (np.arange(H) / H) ** 3 * 20.0
        mine = balanced_bands(cost, 2 * world, 1)[rank::world]
        rendered = band_render_rows(H, mine, 1)
        owned = row_runs(np.nonzero(band_owned_rows(H, mine))[0])
    else:
        rendered = render_rows(H, world, rank, S, 1)
        owned = owned_row_ranges(H, world, rank, S)
    s = Scene((W, H))
    scenes.setup_cornell(s, W, H, 3)
    luts = oracle.luts_from_arrays(dict(np.load(GOLDEN / "bxdf_luts.npz")))
    filt = FilterParams(FILTER_BOX, 1.0, 1.5, 1 / 3, 1 / 3, 3)
    film = np.zeros((H, W, 4), np.float32)
    for seed in range(2):
        fr = s.frame_params(seed)
        pos = np.zeros((H, W, 2), np.float32)
        val = np.zeros((H, W, 4), np.float32)
        for (y0, y1) in row_runs(rendered):
            p, v, _, _ = oracle.render(s.flat(), luts, fr, oracle.WAVEFRONT, rect=(0, y0, W, y1 - y0), threads=1)
            pos[y0:y1], val[y0:y1] = p[y0:y1], v[y0:y1]
        for (r0, r1) in owned:
            oracle.sample_convolution(filt, pos, val, film, rows=(r0, r1))
    t = torch.from_numpy(film)
    dist.reduce(t, dst=0, op=dist.ReduceOp.SUM)
    if rank == 0:
        np.save(os.path.join(out_dir, "film_reduced.npy"), t.numpy())
    dist.destroy_process_group()


@pytest.mark.parametrize("mode", ["stripes", "bands"])
def test_gloo_two_rank_film_reduce_is_bit_exact(tmp_path, oracle_mod, golden_luts, mode):
    """Round-robin stripes, and uneven cost-balanced bands (partition.balanced_bands, two per rank):
    the reduce(SUM) of the ranks' films is the one-rank film bit for bit."""
    import torch.multiprocessing as mp
    from directcomputeraytracing_amd import FILTER_BOX, FilterParams, Scene, scenes
    mp.spawn(_worker, args=(2, _free_port(), str(tmp_path), mode), nprocs=2, join=True)
    reduced = np.load(tmp_path / "film_reduced.npy")
    W, H = 96, 80
    s = Scene((W, H))
    scenes.setup_cornell(s, W, H, 3)
    filt = FilterParams(FILTER_BOX, 1.0, 1.5, 1 / 3, 1 / 3, 3)
    ref = np.zeros((H, W, 4), np.float32)
    for seed in range(2):
        p, v, _, _ = oracle_mod.render(s.flat(), golden_luts, s.frame_params(seed), oracle_mod.WAVEFRONT)
        oracle_mod.sample_convolution(filt, p, v, ref)
    assert np.array_equal(reduced.view(np.uint32), ref.view(np.uint32))


def test_bench_world_check_and_launcher_command():
    """bench.py --gpus N: without a launcher it starts its N ranks (torch.distributed.run on
    127.0.0.1, same arguments); under a launcher a world size other than --gpus is refused."""
    import importlib.util
    spec = importlib.util.spec_from_file_location("bench_mod", ROOT / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    assert bench.check_world(1, {}) is None
    assert bench.check_world(8, {}) == "launch"
    assert bench.check_world(8, {"WORLD_SIZE": "8"}) is None
    assert bench.check_world(1, {"WORLD_SIZE": "1"}) is None
    assert "WORLD_SIZE=4" in bench.check_world(8, {"WORLD_SIZE": "4"})
    assert "WORLD_SIZE=2" in bench.check_world(1, {"WORLD_SIZE": "2"})
    cmd = bench.launcher_command(["--gpus", "8", "--steps", "5"], 8, 29555)
    i = cmd.index("torch.distributed.run")
    assert cmd[i - 1] == "-m" and cmd[cmd.index("--nproc-per-node") + 1] == "8"
    assert cmd[cmd.index("--master-addr") + 1] == "127.0.0.1" and cmd[cmd.index("--master-port") + 1] == "29555"
    assert cmd[-4:] == ["--gpus", "8", "--steps", "5"] and cmd[-5].endswith("bench.py")
