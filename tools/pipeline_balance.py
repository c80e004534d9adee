#!/usr/bin/env python3
"""Diagnostic: per-pipeline work of bench.py's concurrent pipelines (one GPU, Cornell 1080p).

Each of the K pipelines renders its rows (partition.stream_partition) ALONE for the same
images, so the times show how evenly the split divides the work (the bench runs them
concurrently; a pipeline that finishes early leaves the other alone on the GPU).

  python tools/pipeline_balance.py [--streams 2] [--stripe 64] [--images 16]
"""
import argparse
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--streams", type=int, default=2)
    ap.add_argument("--stripe", type=int, default=256)
    ap.add_argument("--images", type=int, default=16)
    ap.add_argument("--pool", type=int, default=1 << 25)
    args = ap.parse_args()
    from directcomputeraytracing_amd import Scene, WavefrontPathTracer, scenes
    from directcomputeraytracing_amd.partition import halo_for_radius, stream_partition
    W, H = 1920, 1080
    scene = Scene((W, H))
    scenes.setup_cornell(scene, W, H, 8)
    filt = scene.filter_params()
    halo = max(1, halo_for_radius(filt.radius, H))
    K = args.streams
    out = []
    for s in range(K):
        part = stream_partition(H, 1, 0, K, s, args.stripe)
        t = WavefrontPathTracer(path_pool_size=args.pool // K, iterations_per_render=16)
        t.on_scene_loaded(scene)
        t.set_film_partition(*part, halo)
        t.prepare_images(args.images)
        t.render_images(1000, 2, filt)     # warm-up batch
        t.synchronize()
        t0 = time.perf_counter()
        t.render_images(0, args.images, filt)
        t.synchronize()
        dt = time.perf_counter() - t0
        out.append(dt)
        print(f"pipeline {s}: partition {part} {dt * 1e3 / args.images:.3f} ms/image", flush=True)
        t.destroy()
    print(f"imbalance max/mean {max(out) / (sum(out) / len(out)):.3f}")


if __name__ == "__main__":
    main()
