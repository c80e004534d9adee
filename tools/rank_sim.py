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
    ap.add_argument("--fixed-pool", action="store_true", help="pool // streams per pipeline (no pipeline_pool sizing)")
    args = ap.parse_args()
    from directcomputeraytracing_amd import Scene, WavefrontPathTracer, render_images_concurrently, scenes
    from directcomputeraytracing_amd.partition import halo_for_radius, pipeline_pool, render_rows, stream_partition
    scene = Scene((1920, 1080))
    scenes.setup_cornell(scene, 1920, 1080, 8)
    filt = scene.filter_params()
    base = None
    for n in [int(x) for x in args.gpus.split(",")]:
        times, rays, iters = [], [], []
        for r in range(1 if args.rank0_only else n):
            # the rank's K concurrent pipelines, as bench.py --streams K runs them
            K = max(1, args.streams)
            ts = []
            try:
                for s_ in range(K):
                    part = stream_partition(1080, n, r, K, s_, args.stripe) if (n > 1 or K > 1) else None
                    halo = max(1, halo_for_radius(filt.radius))
                    rows = len(render_rows(1080, *part, halo)) if part is not None else 1080
                    pool = args.pool // K
                    if not args.image_batch and not args.fixed_pool:   # as bench.py sizes it
                        pool = pipeline_pool(pool, rows, 1920, args.steps * n)
                    t = WavefrontPathTracer(path_pool_size=pool, iterations_per_render=16)
                    ts.append(t)
                    t.on_scene_loaded(scene)
                    t.set_image_batch(args.image_batch)
                    if part is not None:
                        t.set_film_partition(*part, halo)
                    t.clear_film()

                def run(first, count):
                    render_images_concurrently(ts, first, count, filt)

                run(10_000, n)
                for t in ts:
                    t.prepare_images(args.steps * n)
                    t.reset_stats()
                t0 = time.perf_counter()
                run(0, args.steps * n)
                times.append((time.perf_counter() - t0) * 1e3 / args.steps)
                cs = [t.counters() for t in ts]
                rays.append(sum(c["extension_rays"] + c["shadow_rays"] for c in cs) / args.steps)
                iters.append(max(c.get("iterations", 0) for c in cs) / args.steps)
            finally:
                for t in ts:
                    t.destroy()
        mx, mean = max(times), sum(times) / len(times)
        base = base or mx
        print(json.dumps({"n_gpus": n, "ms_per_step_max_rank": round(mx, 3), "ms_per_step_mean_rank": round(mean, 3),
                          "weak_efficiency": round(base / mx, 3), "image_batch": args.image_batch, "pool": args.pool, "fixed_pool": args.fixed_pool, "streams": args.streams,
                          "mrays_per_step_mean_rank": round(sum(rays) / len(rays) / 1e6, 3),
                          "ns_per_ray_mean_rank": round(mean * 1e6 / (sum(rays) / len(rays)), 4),
                          "iterations_per_step_mean_rank": round(sum(iters) / len(iters), 2),
                          "ms_per_step_by_rank": [round(x, 3) for x in times],
                          "iterations_per_step_by_rank": [round(x, 2) for x in iters]}), flush=True)


if __name__ == "__main__":
    main()
