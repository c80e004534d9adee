#!/usr/bin/env python3
"""Experiment: K film partitions of one GPU rendered concurrently on K streams.

Each partition is a tracer of its own (path pool / K, own stream and graphs) that
path-traces its stripes (+halo) of every image, exactly like a rank of the N-GPU
film split; the K host threads enqueue concurrently (ctypes releases the GIL), so
the kernels of the K pipelines overlap on the GPU and fill each other's tails. The
partition films sum to the single-tracer film bit for bit.

  python tools/stream_sim.py [--streams 1,2,3,4] [--steps 32] [--check]
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
    ap.add_argument("--streams", default="1,2,3,4")
    ap.add_argument("--steps", type=int, default=32)
    ap.add_argument("--stripe", type=int, default=256)
    ap.add_argument("--pool", type=int, default=1 << 25, help="total path-pool slots, split over the streams")
    ap.add_argument("--check", action="store_true", help="compare the summed film with the 1-stream film")
    ap.add_argument("--world", type=int, default=1, help="emulate rank --rank of an N-GPU film split")
    ap.add_argument("--rank", type=int, default=0)
    args = ap.parse_args()
    import numpy as np
    from directcomputeraytracing_amd import Scene, WavefrontPathTracer, render_images_concurrently, scenes
    from directcomputeraytracing_amd.partition import halo_for_radius, stream_partition
    scene = Scene((1920, 1080))
    scenes.setup_cornell(scene, 1920, 1080, 8)
    filt = scene.filter_params()
    ref_film, base = None, None
    for k in [int(x) for x in args.streams.split(",")]:
        ts = []
        for r in range(k):
            t = WavefrontPathTracer(path_pool_size=args.pool // k, iterations_per_render=16, device=0)
            t.on_scene_loaded(scene)
            if k > 1 or args.world > 1:
                w, v, sh = stream_partition(1080, args.world, args.rank, k, r, args.stripe)
                t.set_film_partition(w, v, sh, max(1, halo_for_radius(filt.radius)))
            ts.append(t)

        def run_all(first, count):
            render_images_concurrently(ts, first, count, filt)

        try:
            for t in ts:
                t.clear_film()
            run_all(10_000, 2)
            for t in ts:
                t.prepare_images(args.steps)
                t.clear_film()
                t.reset_stats()
            t0 = time.perf_counter()
            run_all(0, args.steps)
            el = time.perf_counter() - t0
            rays = sum(t.counters()["extension_rays"] + t.counters()["shadow_rays"] for t in ts)
            film = sum(t.read_film() for t in ts) if args.check else None
        finally:
            for t in ts:
                t.destroy()
        ms = el * 1e3 / args.steps
        base = base or ms
        out = {"streams": k, "ms_per_spp": round(ms, 3), "speedup": round(base / ms, 3),
               "mrays_per_s": round(rays / el / 1e6, 1), "rays_per_spp": int(rays / args.steps)}
        if args.check:
            if ref_film is None:
                ref_film = film
            out["film_bit_exact_vs_1"] = bool(np.array_equal(film.view(np.uint32), ref_film.view(np.uint32)))
        print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
