#!/usr/bin/env python3
"""Weak-scaling rehearsal on one GPU: the per-rank work of bench.py --gpus N, one rank at a time.

At N GPUs a bench step is N images, each rank path-tracing its stripes (+halo) of all N.
Ranks run independently until the final film reduce, so the N-GPU step time is about the
slowest rank's time; this times every rank's share on this one GPU and prints, per N, the
max / mean rank time per step and the implied weak-scaling efficiency vs N = 1.

  python tools/rank_sim.py [--gpus 1,2,4,8] [--steps 8] [--image-batch 0]
"""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", default="1,2,4,8")
    ap.add_argument("--steps", type=int, default=8)
    ap.add_argument("--image-batch", type=int, default=0)
    ap.add_argument("--stripe", type=int, default=256)
    ap.add_argument("--pool", type=int, default=1 << 25)
    ap.add_argument("--streams", type=int, default=2, help="concurrent pipelines per rank (bench.py --streams)")
    ap.add_argument("--rank0-only", action="store_true", help="time rank 0's share only (sweeps)")
    ap.add_argument("--repeats", type=int, default=3, help="timed repeats per rank; its time is their median")
    ap.add_argument("--interleave", action="store_true", help="pipelines split the images of the rank's rows (bench --interleave)")
    ap.add_argument("--bands-per-rank", type=int, default=0, help="interleaved: balanced bands per rank (0 = --streams)")
    ap.add_argument("--calibrate", type=int, default=0,
                    help="calibration rounds: each renders every rank's share once, untimed by the result, and its rank "
                         "times re-cut the bands at equal time (partition.refine_row_cost, bench --calibrate)")
    ap.add_argument("--calib-repeats", type=int, default=3, help="calibration: median of this many runs per rank")
    ap.add_argument("--fixed-pool", action="store_true", help="pool // streams per pipeline (no pipeline_pool sizing)")
    ap.add_argument("--partition", choices=["balanced", "stripes"], default="balanced",
                    help="balanced: equal-cost contiguous bands from the row-cost probe (bench.py's default); "
                         "stripes: round-robin stripes of --stripe rows")
    args = ap.parse_args()
    from directcomputeraytracing_amd import (Scene, make_pipelines, prepare_pipelines, probe_row_cost,
                                             render_images_concurrently, scenes)
    scene = Scene((1920, 1080))
    scenes.setup_cornell(scene, 1920, 1080, 8)
    filt = scene.filter_params()
    row_cost = probe_row_cost(scene) if args.partition == "balanced" else None
    base = None
    from directcomputeraytracing_amd.partition import balanced_bands, halo_for_radius, refine_row_cost
    halo = max(1, halo_for_radius(filt.radius, 1080))

    def rank_bands(cost, n, K):
        B = (args.bands_per_rank or K) if args.interleave else K
        return [balanced_bands(cost, n * B, halo)[r::n] for r in range(n)]

    for n in [int(x) for x in args.gpus.split(",")]:
        times, rays, iters = [], [], []
        cost_n = row_cost
        K = max(1, args.streams)
        ranks = list(range(1 if args.rank0_only else n))

        def build(cost):
            # every rank's K pipelines at once (a few GB each: the 288 GB of HBM hold all eight
            # ranks), so the repeats can go round-robin over the ranks and a slow drift of the
            # GPU's clock lands on every rank alike instead of reading as imbalance
            shares = []
            try:
                for r in ranks:
                    shares.append(make_pipelines(scene, args.pool, streams=K, images=args.steps * n, iterations=16, world=n,
                                                 rank=r, stripe=args.stripe, image_batch=args.image_batch, row_cost=cost,
                                                 fixed_pool=args.fixed_pool, interleave=args.interleave,
                                                 bands_per_rank=args.bands_per_rank))
                for ts in shares:
                    for t in ts:
                        t.clear_film()
                    render_images_concurrently(ts, 10_000, n, filt)
                    prepare_pipelines(ts, args.steps * n)
            except BaseException:
                destroy(shares)
                raise
            return shares

        def destroy(shares):
            for ts in shares:
                for t in ts:
                    t.destroy()

        def time_ranks(shares, first, repeats):
            reps = [[] for _ in shares]
            for _ in range(max(1, repeats)):
                for i, ts in enumerate(shares):
                    for t in ts:
                        t.clear_film()
                        t.reset_stats()
                    t0 = time.perf_counter()
                    render_images_concurrently(ts, first, args.steps * n, filt)
                    reps[i].append((time.perf_counter() - t0) * 1e3 / args.steps)
            return [sorted(x)[len(x) // 2] for x in reps]   # (bench.py: the median of its repeats)

        cost_n = row_cost
        for _round in range(args.calibrate if (row_cost is not None and n > 1 and not args.rank0_only) else 0):
            # a calibration round (bench.py --calibrate): the median rank times of the prepared
            # workload on other seeds re-cut the bands at equal time
            shares = build(cost_n)
            try:
                calib = time_ranks(shares, 30_000, args.calib_repeats)
            finally:
                destroy(shares)
            cost_n = refine_row_cost(cost_n, rank_bands(cost_n, n, K), calib, halo)
        shares = build(cost_n)
        try:
            times = time_ranks(shares, 0, args.repeats)
            for ts in shares:
                cs = [t.counters() for t in ts]
                rays.append(sum(c["extension_rays"] + c["shadow_rays"] for c in cs) / args.steps)
                iters.append(max(c.get("iterations", 0) for c in cs) / args.steps)
        finally:
            destroy(shares)
        mx, mean = max(times), sum(times) / len(times)
        base = base or mx
        print(json.dumps({"n_gpus": n, "ms_per_step_max_rank": round(mx, 3), "ms_per_step_mean_rank": round(mean, 3),
                          "weak_efficiency": round(base / mx, 3), "repeats": args.repeats, "partition": args.partition, "interleave": args.interleave, "bands_per_rank": args.bands_per_rank, "calibrate": args.calibrate, "image_batch": args.image_batch, "pool": args.pool, "fixed_pool": args.fixed_pool, "streams": args.streams,
                          "mrays_per_step_mean_rank": round(sum(rays) / len(rays) / 1e6, 3),
                          "ns_per_ray_mean_rank": round(mean * 1e6 / (sum(rays) / len(rays)), 4),
                          "iterations_per_step_mean_rank": round(sum(iters) / len(iters), 2),
                          "ms_per_step_by_rank": [round(x, 3) for x in times],
                          "iterations_per_step_by_rank": [round(x, 2) for x in iters]}), flush=True)


if __name__ == "__main__":
    main()
