#!/usr/bin/env python3
"""Headline benchmark: Mrays/s and ms/spp, Cornell box 1920x1080, 8-bounce wavefront.

A *step* is N one-sample-per-pixel images of the full film (N = number of GPUs;
frame seed = image index), rendered by the wavefront pipeline and convolved
into the fp32 film. Each rank renders its round-robin stripes (+halo) of every
image, so per-GPU work per step is one full image: weak scaling. ``--gpus N``
> 1 is launched by torch.distributed.run; one RCCL reduce of the RGBA32F film
closes the timed region.

``--config coffee|spaceship|lamp`` runs BASELINE.json's other configs (procedural
scenes, their resolutions) through the same path, on 1 or N GPUs.

Prints ONE JSON line (rank 0). Besides the contract fields it carries
``roofline`` (the merged EXTENSION+SHADOW cast launch: algorithmic bytes per
launch / HIP-event launch time against the MI355X HBM peak, next to the
PMC-measured HBM bytes of the same launches when a profile of this workload is
committed) and ``cpu_baseline`` (the oracle's scalar
MegakernelPathTracing restatement on this host's cores, bounded sample).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

HBM_PEAK_GBS = 8000.0          # MI355X HBM3E, /opt/skills/guides/MI355X_MICROARCH.md
EXT_RAY_BYTES = 4 + 32 + 20    # queue index + SRay + SRayHit
NODE_BYTES, TRI_BYTES, BLAS_BYTES = 32, 48, 56
SHADOW_RAY_BYTES = 4 + 32 + 4 + 4
CONTROL_BYTES, MATERIAL_BYTES, NEW_PATH_BYTES = 92, 600, 88   # per path-iteration / new path
FILM_BYTES_BASE, FILM_BYTES_PER_TAP = 32, 24                  # SampleConvolution: 24 B per window tap + 32


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=64, help="timed images (1 spp each); configs[1] is 64 spp")
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--width", type=int, default=1920)
    ap.add_argument("--height", type=int, default=1080)
    ap.add_argument("--bounces", type=int, default=8)
    ap.add_argument("--config", default="cornell", choices=["cornell", "coffee", "spaceship", "lamp"],
                    help="BASELINE.json configs[1..4]; the headline (and default) is cornell = configs[1]")
    ap.add_argument("--scene-dir", default="/tmp/dcrt_scenes", help="where the procedural config scenes are written")
    ap.add_argument("--snapshot-spp", type=int, default=0,
                    help="progressive: reduce the film onto rank 0 every K images (configs[4]); 0 = once at the end")
    ap.add_argument("--pool", type=int, default=0,
                    help="path pool slots (0: 2^24 at 1080p = 8 images in flight, one drain per batch; 2^26 at 4K)")
    ap.add_argument("--iterations", type=int, default=16, help="wavefront iterations per graph launch")
    ap.add_argument("--stripe", type=int, default=64, help="film stripe height for N>1")
    ap.add_argument("--streams", type=int, default=2,
                    help="concurrent wavefront pipelines per GPU (film partitions on their own streams)")
    ap.add_argument("--image-batch", type=int, default=0, help="images per wavefront batch (0 = automatic)")
    ap.add_argument("--roofline-images", type=int, default=0,
                    help="images of the roofline leg (0 = the timed images, so its launches are the timed region's)")
    ap.add_argument("--dist-backend", default="nccl", help="nccl (= RCCL over xGMI) or gloo (CPU reduce, for tests)")
    ap.add_argument("--save-film", default=None, help="rank 0 writes the reduced RGBA32F film (.npy)")
    ap.add_argument("--mode", choices=["wavefront", "megakernel"], default="wavefront",
                    help="A/B: the reference's two tracers (the contract line is the wavefront)")
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="target CPU-baseline sample duration")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--traffic-json", default=None,
                    help="PMC summary from tools/pmc_traffic.py (default: the newest profiles/r*_pmc_traffic*.json "
                         "whose recorded workload is this run's)")
    return ap.parse_args()


def cpu_baseline(scene, luts_arrays, seconds: float, label: str = "1920x1080 8-bounce Cornell") -> dict:
    """Oracle megakernel (MegakernelPathTracing.hlsl restated in C) on host cores, bounded."""
    import oracle  # cpu_baseline leg only
    threads = max(1, min(int(os.environ.get("OMP_NUM_THREADS", "16") or 16), os.cpu_count() or 1, 16))
    luts = oracle.luts_from_arrays(luts_arrays)
    flat = scene.flat()
    fr = scene.frame_params(0)
    W, H = fr.resolution[0], fr.resolution[1]
    # whole 1-spp images (seeds 0, 1, ...) until about `seconds` of CPU time; if one
    # image would take far longer, a centred band of rows sized from a 16-row probe
    t0 = time.perf_counter()
    oracle.render(flat, luts, fr, oracle.MEGAKERNEL, rect=(0, (H - 16) // 2, W, 16), threads=threads)
    rate = 16 / max(time.perf_counter() - t0, 1e-6)
    band = int(min(H, max(16, rate * seconds)))
    rays, elapsed, images = 0, 0.0, 0
    while elapsed < seconds:
        fr_s = scene.frame_params(images)
        t0 = time.perf_counter()
        _, _, _, c = oracle.render(flat, luts, fr_s, oracle.MEGAKERNEL, rect=(0, (H - band) // 2, W, band),
                                   threads=threads)
        elapsed += time.perf_counter() - t0
        rays += c["extension_rays"] + c["shadow_rays"]
        images += 1
        if band < H:
            break
    done_rows = band * images
    mrays = rays / elapsed / 1e6
    return {"value": round(mrays, 3), "unit": "Mrays/s", "cores": threads, "kind": "port",
            "sample": f"oracle megakernel (scalar C restatement of MegakernelPathTracing.hlsl), {W}x{done_rows} "
                      f"rows ({images} image(s) of {band} rows, seeds 0..{images - 1}) of the {label} "
                      f"image at 1 spp, {elapsed:.1f} s",
            "ms_per_spp_extrapolated": round(elapsed * 1e3 * H / done_rows, 1)}


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    device = local_rank
    if world > 1:
        import torch
        import torch.distributed as dist
        device = local_rank % max(1, torch.cuda.device_count())
        torch.cuda.set_device(device)
        if args.dist_backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", device))
        else:
            dist.init_process_group(args.dist_backend)

    if args.snapshot_spp and world == 1:
        # torch (its own HIP runtime) must own the device before libdcrt's runtime does
        import torch
        torch.cuda.set_device(device)

    import numpy as np
    from directcomputeraytracing_amd import Scene, WavefrontPathTracer, render_images_concurrently, scenes
    luts_arrays = dict(np.load(ROOT / "tests" / "golden" / "bxdf_luts.npz"))

    scene = Scene((args.width, args.height))
    if args.config == "cornell":
        scenes.setup_cornell(scene, args.width, args.height, args.bounces)
        workload = (f"cornell_box_obj {args.width}x{args.height}, {{spp}} spp ({world} spp/step, film stripes across "
                    f"{world} GPU(s)), {args.bounces} bounces, wavefront, point light")
    else:
        desc = scenes.setup_config(scene, args.config, args.scene_dir)
        args.width, args.height = scene.resolution
        workload = f"{desc}, {{spp}} spp ({world} spp/step, film stripes across {world} GPU(s)), wavefront"
    args.pool = args.pool or scenes.default_pool(args.width, args.height)
    filt = scene.filter_params()
    from directcomputeraytracing_amd.partition import halo_for_radius, pipeline_pool, render_rows, stream_partition
    halo = max(1, halo_for_radius(filt.radius, args.height))

    def make_tracer(pool, part):
        t = WavefrontPathTracer(path_pool_size=pool, iterations_per_render=args.iterations, device=device)
        t.on_scene_loaded(scene)
        t.set_mode(args.mode)
        t.set_image_batch(args.image_batch)
        if part is not None:
            t.set_film_partition(*part, halo)
        return t

    # K concurrent pipelines per GPU (--streams): tracer s renders the rank's stripes dealt
    # to it (partition.stream_partition), on its own stream, from its own host thread; the
    # K films have disjoint supports and are summed on the device (add_film_device).
    K = max(1, args.streams)
    tracers = []
    for s_ in range(K):
        part = stream_partition(args.height, world, rank, K, s_, args.stripe) if (K > 1 or world > 1) else None
        # (a pool just short of a whole number of batches grows by <= 5 %: one drain less)
        rows = len(render_rows(args.height, *part, halo)) if part is not None else args.height
        pool = pipeline_pool(args.pool // K, rows, args.width, args.steps * world) if not args.image_batch else args.pool // K
        tracers.append(make_tracer(pool, part))
    tracer = tracers[0]

    def render_all(first, count):
        render_images_concurrently(tracers, first, count, filt)

    def barrier_sync():
        for t in tracers:
            t.synchronize()
        if dist is not None:
            import torch
            torch.cuda.synchronize()
            dist.barrier()

    def combine_films():
        # the K pipelines' films into tracer 0's (disjoint supports: bit-exact sum)
        for t in tracers[1:]:
            t.synchronize()
            tracer.add_film_device(t.film_device_ptr())

    film_buf = None
    on_device = args.dist_backend == "nccl"
    if dist is not None:
        import torch
        film_buf = torch.empty(args.width * args.height * 4, dtype=torch.float32, device="cuda" if on_device else "cpu")

    snap_dev = snap_tmp = None
    if args.snapshot_spp:
        import torch
        n4 = args.width * args.height * 4
        snap_dev = film_buf if (film_buf is not None and on_device) else torch.empty(n4, dtype=torch.float32, device="cuda")
        snap_tmp = torch.empty(n4, dtype=torch.float32, device="cuda") if K > 1 else None

    def snapshot_film():
        # the rank's film = sum of its pipelines' films (disjoint supports), then the reduce
        import torch
        for t in tracers:
            t.synchronize()
        tracers[0].copy_film_device(snap_dev.data_ptr())
        for t in tracers[1:]:
            t.copy_film_device(snap_tmp.data_ptr())
            snap_dev.add_(snap_tmp)
            # the next pipeline's copy (on its own stream) overwrites snap_tmp: wait for the add
            torch.cuda.synchronize()
        torch.cuda.synchronize()
        if dist is not None:
            if not on_device:
                film_buf.copy_(snap_dev.cpu())
            dist.reduce(film_buf, dst=0, op=dist.ReduceOp.SUM)

    def reduce_film():
        # the one data-path collective: SUM of the disjointly-supported stripe films on rank 0
        if on_device:
            tracer.copy_film_device(film_buf.data_ptr())
        else:
            import torch
            film_buf.copy_(torch.from_numpy(tracer.read_film().reshape(-1)))
        dist.reduce(film_buf, dst=0, op=dist.ReduceOp.SUM)

    # warmup (also builds the graphs)
    for t in tracers:
        t.clear_film()
    if args.warmup:
        render_all(10_000, args.warmup)
    images = args.steps * world            # weak scaling: each step is one image per GPU-equivalent
    for t in tracers:
        t.prepare_images(images)           # sample textures of the timed batches + graph: not timed work
        t.clear_film()
        t.reset_stats()
    barrier_sync()
    t0 = time.perf_counter()
    snapshots = bool(args.snapshot_spp and args.snapshot_spp < images)
    if snapshots:
        # progressive rendering (configs[4]): every K images the films so far are summed
        # over the pipelines and reduced onto rank 0 (a preview); the tracers' films keep
        # accumulating, so the last snapshot is the whole render
        done = 0
        while done < images:
            n = min(args.snapshot_spp, images - done)
            render_all(done, n)
            done += n
            snapshot_film()
    else:
        render_all(0, images)
        combine_films()
        if dist is not None:
            reduce_film()
    barrier_sync()
    elapsed = time.perf_counter() - t0
    rays = 0
    for t in tracers:
        c = t.counters()
        rays += c["extension_rays"] + c["shadow_rays"]

    if dist is not None:
        import torch
        tt = torch.tensor([elapsed, float(rays)], dtype=torch.float64, device="cuda" if on_device else "cpu")
        tmax = tt[:1].clone()
        dist.all_reduce(tmax, op=dist.ReduceOp.MAX)
        tsum = tt[1:].clone()
        dist.all_reduce(tsum, op=dist.ReduceOp.SUM)
        elapsed, rays = float(tmax.item()), float(tsum.item())

    if args.save_film and rank == 0:
        # the reduced film (N > 1), the last snapshot (one rank, snapshots taken), else tracer 0's
        # film, which combine_films made the sum of the rank's pipelines
        if dist is not None:
            film = film_buf.cpu().numpy()
        elif snapshots:
            film = snap_dev.cpu().numpy()
        else:
            film = tracer.read_film()
        np.save(args.save_film, film.reshape(args.height, args.width, 4))

    # ---- roofline leg: same workload (seeds 0..R-1), counters then HIP-event timing, on
    # ONE pipeline (the rank's whole partition, as with --streams 1): a kernel's duration
    # is only its own when no other pipeline's kernels share the GPU
    R = max(1, args.roofline_images or images)
    if K > 1:
        for t in tracers:
            t.destroy()
        tracer = make_tracer(args.pool, (world, rank, args.stripe) if world > 1 else None)
    tracer.set_instrumentation(True, False)
    tracer.reset_stats()
    tracer.render_images(0, R, filt)
    st = tracer.traversal_stats()
    cr = tracer.counters()
    tracer.set_instrumentation(False, True)
    tracer.reset_stats()
    tracer.render_images(0, R, filt)
    tm = tracer.traversal_stats()
    tracer.set_instrumentation(False, False)
    ext_bytes = (EXT_RAY_BYTES * cr["extension_rays"] + NODE_BYTES * st["ext_node_visits"]
                 + TRI_BYTES * st["ext_triangle_tests"] + BLAS_BYTES * st["ext_blas_entries"])
    shadow_bytes = (SHADOW_RAY_BYTES * cr["shadow_rays"] + NODE_BYTES * st["shadow_node_visits"]
                    + TRI_BYTES * st["shadow_triangle_tests"] + BLAS_BYTES * st["shadow_blas_entries"])
    # the timed launch is the merged EXTENSION+SHADOW cast kernel unless DCRT_SPLIT_CASTS=1
    merged = os.environ.get("DCRT_SPLIT_CASTS", "0") in ("", "0")
    cast_bytes = ext_bytes + shadow_bytes if merged else ext_bytes
    launches = max(1, tm["ext_launches"])
    avg_ms = tm["ext_kernel_ms"] / launches
    bytes_per_launch = cast_bytes / launches
    achieved = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    # measured HBM traffic of the same cast launches: a committed rocprofv3 PMC summary of
    # THIS workload (tools/profile.sh + tools/pmc_traffic.py record the workload they profiled),
    # never a profile of another image count, pool or scene
    # whole-pipeline roofline ("and for the whole pipeline"): the reference's
    # algorithmic bytes of every stage for the timed images (cast terms as above, CONTROL +
    # MATERIAL per path-iteration = per extension ray, NEW_PATH per new path, the film pass
    # per pixel x image), from the roofline leg's counts of the same images, over the timed
    # region's wall time (max over ranks), per GPU
    film_bytes = FILM_BYTES_BASE + FILM_BYTES_PER_TAP * (2 * int(filt.radius + 0.5) + 1) ** 2
    pipe_bytes_R = (ext_bytes + shadow_bytes + (CONTROL_BYTES + MATERIAL_BYTES) * cr["extension_rays"]
                    + NEW_PATH_BYTES * cr["new_paths"] + film_bytes * args.width * args.height * R / world)
    pipe_achieved = pipe_bytes_R * (images / R) / elapsed / 1e9
    workload_key = {"config": args.config, "resolution": [args.width, args.height], "images": R,
                    "path_pool": args.pool, "world": world}
    traffic, traffic_src = None, "no committed PMC profile of this workload"
    cands = [Path(args.traffic_json)] if args.traffic_json else \
        sorted((ROOT / "profiles").glob("r*_pmc_traffic*.json"), reverse=True)
    for tj in cands:
        try:
            d = json.loads(tj.read_text())
        except Exception:
            continue
        if d.get("workload") == workload_key and d.get("ext_hbm_bytes_per_launch"):
            traffic = d["ext_hbm_bytes_per_launch"]
            traffic_src = (f"{tj.relative_to(ROOT) if tj.is_relative_to(ROOT) else tj}: rocprofv3 PMC, "
                           f"FETCH_SIZE x2 + WRITE_SIZE per cast launch, same workload")
            break

    result = {
        "metric": ("Mrays/s and ms/spp at 1920x1080, 8-bounce wavefront" if args.config == "cornell"
                   else f"Mrays/s and ms/spp at {args.width}x{args.height}, {args.config} config, wavefront"),
        "value": round(rays / elapsed / 1e6, 2),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
        "ms_per_spp": round(elapsed * 1e3 / images, 3),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": workload.format(spp=images), "name": args.config,
                   "resolution": [args.width, args.height], "spp": images,
                   "max_bounce": args.bounces if args.config == "cornell" else scene.frame_params(0).max_bounce_count,
                   "path_pool": args.pool, "streams_per_gpu": K, "snapshot_spp": args.snapshot_spp or images,
                   "parallelism": (f"film stripes x{world}" if world > 1 else "single GPU")
                                  + (f", {K} concurrent pipelines per GPU" if K > 1 else ""),
                   "rays": int(rays)},
        "roofline": {"bound": "hbm",
                     "basis": "algorithmic bytes: the reference's traversal counts (node visits, triangle tests, "
                              "BLAS entries, from the instrumented kernel) x SURVEY 8(d)'s bytes per unit, "
                              "wherever the bytes are served from (LDS scene cache, L1, L2, MALL or HBM)",
                     "kernel": "cast_kernel (EXTENSION_RAY_CAST + SHADOW_RAY_CAST, one launch)" if merged
                               else "extension_kernel (EXTENSION_RAY_CAST)",
                     "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                     "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
                     "traffic_source": traffic_src,
                     "hbm_measured": None if traffic is None else
                     {"achieved": round(traffic / (avg_ms * 1e-3) / 1e9, 1),
                      "frac": round(traffic / (avg_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4)},
                     "bytes_per_launch": int(bytes_per_launch), "avg_launch_us": round(avg_ms * 1e3, 2),
                     "launches": int(launches), "images": R,
                     "per_ext_ray": {"nodes": st["ext_node_visits"] / max(1, cr["extension_rays"]),
                                     "tris": st["ext_triangle_tests"] / max(1, cr["extension_rays"]),
                                     "blas": st["ext_blas_entries"] / max(1, cr["extension_rays"])},
                     "per_shadow_ray": {"nodes": st["shadow_node_visits"] / max(1, cr["shadow_rays"]),
                                        "tris": st["shadow_triangle_tests"] / max(1, cr["shadow_rays"]),
                                        "blas": st["shadow_blas_entries"] / max(1, cr["shadow_rays"])}},
        "pipeline_roofline": {"bound": "hbm", "achieved": round(pipe_achieved, 1), "peak": HBM_PEAK_GBS,
                              "unit": "GB/s", "frac": round(pipe_achieved / HBM_PEAK_GBS, 4),
                              "bytes_per_spp": int(pipe_bytes_R / R),
                              "basis": "per GPU: algorithmic bytes of cast + CONTROL (92 B) + MATERIAL (600 B) per "
                                       "path-iteration + NEW_PATH (88 B) per new path + film pass per pixel-image "
                                       "(SURVEY 8(d)) over the timed region's wall time"},
        "cpu_baseline": None,
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        label = "1920x1080 8-bounce Cornell" if args.config == "cornell" else f"{args.config} config"
        result["cpu_baseline"] = cpu_baseline(scene, luts_arrays, args.cpu_seconds, label)
    if rank == 0:
        print(json.dumps(result), flush=True)
    tracer.destroy()
    if dist is not None:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
