#!/usr/bin/env python3
"""Secondary benchmark: Mrays/s, ms/spp and the EXTENSION_RAY_CAST roofline on every
BASELINE.json config that fits one GPU (configs[1..4]; the multi-GPU film split of
configs 4/5 is exercised by bench.py --gpus N). Scenes are generated procedurally
(deterministic) into --scene-dir. Prints one JSON line per config.

  python tools/bench_configs.py [--spp K] [--configs cornell,coffee,spaceship,spaceship_close,lamp]
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent.parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0


def setup(name, scene_dir: Path, small: bool):
    from directcomputeraytracing_amd import Scene, scenes
    s = Scene((1920, 1080))
    return s, scenes.setup_config(s, name, scene_dir, small)


def run(name, args):
    from directcomputeraytracing_amd import WavefrontPathTracer, render_images_concurrently
    t0 = time.perf_counter()
    scene, desc = setup(name, Path(args.scene_dir), args.small)
    load_s = time.perf_counter() - t0
    W, H = scene.resolution
    # several images in flight (an image batch), so each batch drains once: 8 images at 1080p, 8 at 4K
    from directcomputeraytracing_amd import scenes
    pool = args.pool or scenes.default_pool(W, H)
    filt = scene.filter_params()
    # the timed images on --streams concurrent pipelines (film bands, bench.py --streams)
    from directcomputeraytracing_amd.partition import halo_for_radius, stream_partition
    K = max(1, args.streams)
    subs = []
    for s_ in range(K):
        t = WavefrontPathTracer(path_pool_size=pool // K, iterations_per_render=16)
        t.on_scene_loaded(scene)
        if K > 1:
            w, v, sh = stream_partition(H, 1, 0, K, s_, 64)
            t.set_film_partition(w, v, sh, max(1, halo_for_radius(filt.radius)))
        subs.append(t)

    def render_all(first, count):
        render_images_concurrently(subs, first, count, filt)

    try:
        for t in subs:
            t.clear_film()
        render_all(10_000, args.warmup)
        for t in subs:
            t.prepare_images(args.spp)
            t.reset_stats()
        t0 = time.perf_counter()
        render_all(0, args.spp)
        el = time.perf_counter() - t0
        rays = sum(t.counters()["extension_rays"] + t.counters()["shadow_rays"] for t in subs)
    finally:
        for t in subs:
            t.destroy()
    tr = WavefrontPathTracer(path_pool_size=pool, iterations_per_render=16)
    try:
        tr.on_scene_loaded(scene)
        # roofline leg (same seeds): counts from the instrumented casts, time from HIP events
        tr.set_instrumentation(True, False)
        tr.reset_stats()
        tr.render_images(0, args.spp, filt)
        st = tr.traversal_stats()
        cr = tr.counters()
        tr.set_instrumentation(False, True)
        tr.reset_stats()
        tr.render_images(0, args.spp, filt)
        tm = tr.traversal_stats()
        tr.set_instrumentation(False, False)
        ext_bytes = (56 * cr["extension_rays"] + 32 * st["ext_node_visits"] + 48 * st["ext_triangle_tests"]
                     + 56 * st["ext_blas_entries"])
        shadow_bytes = (44 * cr["shadow_rays"] + 32 * st["shadow_node_visits"] + 48 * st["shadow_triangle_tests"]
                        + 56 * st["shadow_blas_entries"])
        # the timed launch is the merged EXTENSION+SHADOW cast kernel (as in bench.py)
        achieved = (ext_bytes + shadow_bytes) / (tm["ext_kernel_ms"] * 1e-3) / 1e9
        info = scene.bvh_info()
        return {"config": name, "workload": desc, "resolution": [W, H], "spp": args.spp, "path_pool": pool, "streams": K,
                "value": round(rays / el / 1e6, 1), "unit": "Mrays/s", "ms_per_spp": round(el * 1e3 / args.spp, 2),
                "rays_per_spp": int(rays / args.spp), "triangles_bvh_nodes": info["total_nodes"],
                "scene_load_s": round(load_s, 2),
                "roofline": {"kernel": "cast_kernel (EXTENSION_RAY_CAST + SHADOW_RAY_CAST)", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                             "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                             "avg_launch_us": round(tm["ext_kernel_ms"] * 1e3 / max(1, tm["ext_launches"]), 1),
                             "nodes_per_ray": round(st["ext_node_visits"] / max(1, cr["extension_rays"]), 2),
                             "tris_per_ray": round(st["ext_triangle_tests"] / max(1, cr["extension_rays"]), 2),
                             "blas_per_ray": round(st["ext_blas_entries"] / max(1, cr["extension_rays"]), 2),
                             "shadow_nodes_per_ray": round(st["shadow_node_visits"] / max(1, cr["shadow_rays"]), 2)}}
    finally:
        tr.destroy()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spp", type=int, default=8)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--configs", default="cornell,coffee,spaceship,spaceship_close,lamp")
    ap.add_argument("--scene-dir", default="/tmp/dcrt_scenes")
    ap.add_argument("--streams", type=int, default=2, help="concurrent pipelines (bench.py --streams)")
    ap.add_argument("--pool", type=int, default=0, help="path pool slots (0: scenes.default_pool: 2^25 at 1080p, 2^26 at 4K)")
    ap.add_argument("--small", action="store_true", help="small meshes (CI smoke)")
    args = ap.parse_args()
    for name in args.configs.split(","):
        print(json.dumps(run(name, args)), flush=True)


if __name__ == "__main__":
    main()
