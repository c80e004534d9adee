#!/usr/bin/env python3
"""Headline benchmark: Mrays/s and ms/spp, Cornell box 1920x1080, 8-bounce wavefront.

A *step* is N one-sample-per-pixel images of the full film (N = number of GPUs;
frame seed = image index), rendered by the wavefront pipeline and convolved
into the fp32 film. Each rank renders its round-robin stripes (+halo) of every
image, so per-GPU work per step is one full image: weak scaling. ``--gpus N``
> 1 is launched by torch.distributed.run (started here as a child process when
the driver did not launch the ranks itself); one RCCL reduce of the RGBA32F film
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

import numpy as np

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
    ap.add_argument("--config", default="cornell", choices=["cornell", "coffee", "spaceship", "lamp", "spaceship_close"],
                    help="BASELINE.json configs[1..4]; the headline (and default) is cornell = configs[1]")
    ap.add_argument("--scene-dir", default="/tmp/dcrt_scenes", help="where the procedural config scenes are written")
    ap.add_argument("--no-multiscattering", action="store_true",
                    help="coffee: keep the loaders' Kulla-Conty flag (off) instead of configs[2]'s multiscattering (A/B)")
    ap.add_argument("--snapshot-spp", type=int, default=0,
                    help="progressive: reduce the film onto rank 0 every K images (configs[4]); 0 = once at the end")
    ap.add_argument("--pool", type=int, default=0,
                    help="path pool slots (0: 2^24 per pipeline at 1080p = 8 images in flight each; 2^26 at 4K)")
    ap.add_argument("--iterations", type=int, default=16, help="wavefront iterations per graph launch")
    ap.add_argument("--stripe", type=int, default=256,
                    help="film stripe height for N>1 (256: fewer halo rows than 64, -1 to -2 %% per rank at N = 2 / 4, profiles/r05_ab_pool.txt)")
    ap.add_argument("--partition", choices=["balanced", "stripes"], default="balanced",
                    help="film tiling over ranks and pipelines: balanced = contiguous equal-cost bands cut from the "
                         "row-cost probe (rays per film row of one probe image, identical on every rank); stripes = "
                         "equal-height round-robin stripes of --stripe rows")
    ap.add_argument("--streams", type=int, default=0,
                    help="concurrent wavefront pipelines per GPU (film partitions on their own streams); 0: 3 for "
                         "Cornell at every N, 2 otherwise (profiles/r05_ab_pool.txt, profiles/r06_rank_sim_partition.txt)")
    ap.add_argument("--interleave", choices=["auto", "on", "off"], default="auto",
                    help="on: the GPU's pipelines share the rank's rows and split the images (no halo between them, "
                         "equal work per pipeline); off: each pipeline its own band; auto: on for N > 1")
    ap.add_argument("--bands-per-rank", type=int, default=1,
                    help="interleaved: cost-balanced bands per rank, dealt round-robin over the ranks")
    ap.add_argument("--calibrate", type=int, default=1,
                    help="N > 1 balanced: calibration rounds, each an untimed render of the timed workload whose "
                         "per-rank times re-cut the bands at equal time (partition.refine_row_cost); 0 = the probe's "
                         "ray counts alone")
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
    ap.add_argument("--repeats", type=int, default=5,
                    help="timed repeats of the K steps; value is the median (SURVEY 8(d): median of 5 after warm-up)")
    ap.add_argument("--spaceship-spp", type=int, default=16,
                    help="configs[3] leg of the default Cornell run: spaceship 4K images (0 = skip); 16 = four "
                         "batches per pipeline, the steady state of configs[3]'s 128 spp (4 is one batch: its "
                         "ramp and drain alone)")
    return ap.parse_args()


def host_cpus() -> dict:
    """The host the CPU baseline runs on: nproc (= std::thread::hardware_concurrency()),
    the CPUs this process may use (affinity, cgroup quota) and the CPU model."""
    nproc = os.cpu_count() or 1
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = nproc
    quota = None
    try:
        q, period = Path("/sys/fs/cgroup/cpu.max").read_text().split()[:2]
        if q != "max":
            quota = float(q) / float(period)
    except (OSError, ValueError):
        pass
    model = None
    try:
        model = next((l.split(":", 1)[1].strip() for l in Path("/proc/cpuinfo").read_text().splitlines()
                      if l.startswith("model name")), None)
    except OSError:
        pass
    usable = affinity if quota is None else max(1, min(affinity, int(quota)))
    return {"nproc": nproc, "affinity": affinity, "cgroup_cpus": quota, "usable": usable, "model": model}


def cpu_baseline(scene, luts_arrays, seconds: float, label: str = "1920x1080 8-bounce Cornell") -> dict:
    """Oracle megakernel (MegakernelPathTracing.hlsl restated in C) on host cores, bounded.
    Threads: every CPU this process may run on (hardware_concurrency() limited only by the
    container's affinity / cgroup CPU quota, which caps what more threads could use)."""
    import oracle  # cpu_baseline leg only
    host = host_cpus()
    threads = host["usable"]
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
    # BASELINE configs[0], reported in full: the Cornell OBJ at 128x128,
    # 1 spp, maxBounce 2 -- the host scene load + BVH build (C++, this package) and the scalar
    # megakernel on the same threads; median of 5 after one warm-up
    from directcomputeraytracing_amd import Scene, scenes
    builds, renders, c0_rays = [], [], 0
    for rep in range(6):
        t0 = time.perf_counter()
        s0 = Scene((128, 128))
        scenes.setup_cornell(s0, 128, 128, 2)
        f0 = s0.flat()
        t1 = time.perf_counter()
        _, _, _, c = oracle.render(f0, luts, s0.frame_params(0), oracle.MEGAKERNEL, threads=threads)
        t2 = time.perf_counter()
        if rep:
            builds.append(t1 - t0)
            renders.append(t2 - t1)
        c0_rays = c["extension_rays"] + c["shadow_rays"]
    r0 = float(np.median(renders))
    config0 = {"workload": "configs[0]: Cornell box OBJ 128x128, 1 spp, maxBounce 2, CPU BVH build + scalar megakernel",
               "mrays_per_s": round(c0_rays / r0 / 1e6, 3), "ms_per_spp": round(r0 * 1e3, 3),
               "scene_load_and_bvh_ms": round(float(np.median(builds)) * 1e3, 3), "rays": int(c0_rays),
               "threads": threads}
    return {"value": round(mrays, 3), "unit": "Mrays/s", "cores": threads, "kind": "port", "config0": config0,
            "nproc": host["nproc"], "cpu_model": host["model"], "affinity_cpus": host["affinity"],
            "cgroup_cpus": host["cgroup_cpus"],
            "sample": f"oracle megakernel (scalar C restatement of MegakernelPathTracing.hlsl), {W}x{done_rows} "
                      f"rows ({images} image(s) of {band} rows, seeds 0..{images - 1}) of the {label} "
                      f"image at 1 spp, {elapsed:.1f} s, {threads} threads",
            "ms_per_spp_extrapolated": round(elapsed * 1e3 * H / done_rows, 1)}


def free_port() -> int:
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launcher_command(argv, gpus: int, port: int) -> list:
    """`bench.py --gpus N` started without a launcher: the torch.distributed.run command that
    starts its N ranks (one process per GPU, rendezvous on 127.0.0.1), same arguments."""
    return [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(gpus),
            "--master-addr", "127.0.0.1", "--master-port", str(port), str(Path(__file__).resolve()), *argv]


def check_world(gpus: int, env=os.environ):
    """None when this process is a rank of a --gpus-sized job (or a lone --gpus 1 process);
    "launch" when --gpus N > 1 was given without a launcher (start the ranks as children);
    otherwise the error message (the launcher's world size differs from --gpus)."""
    world = env.get("WORLD_SIZE")
    if world is None:
        return "launch" if gpus > 1 else None
    if int(world) != gpus:
        return f"bench.py: --gpus {gpus} but WORLD_SIZE={world}: the launcher started a different number of ranks"
    return None


def main():
    args = parse()
    state = check_world(args.gpus)
    if state == "launch":
        # Nothing here has touched the GPU (no torch, no libdcrt yet): start the ranks as a
        # CHILD process tree (never an exec) and relay rank 0's JSON line and the exit code.
        import subprocess
        cmd = launcher_command(sys.argv[1:], args.gpus, free_port())
        print("bench.py: launching " + " ".join(cmd), file=sys.stderr, flush=True)
        sys.exit(subprocess.run(cmd).returncode)
    if state is not None:
        print(state, file=sys.stderr, flush=True)
        sys.exit(2)
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
    from directcomputeraytracing_amd import (Scene, WavefrontPathTracer, make_pipelines, prepare_pipelines,
                                             render_images_concurrently, scenes)
    luts_arrays = dict(np.load(ROOT / "tests" / "golden" / "bxdf_luts.npz"))

    scene = Scene((args.width, args.height))
    if args.config == "cornell":
        scenes.setup_cornell(scene, args.width, args.height, args.bounces)
        workload = (f"cornell_box_obj {args.width}x{args.height}, {{spp}} spp ({world} spp/step, film stripes across "
                    f"{world} GPU(s)), {args.bounces} bounces, wavefront, point light")
    else:
        desc = scenes.setup_config(scene, args.config, args.scene_dir, multiscattering=not args.no_multiscattering)
        args.width, args.height = scene.resolution
        workload = f"{desc}, {{spp}} spp ({world} spp/step, film stripes across {world} GPU(s)), wavefront"
    # pipelines per GPU: three for Cornell at every N (its LDS-resident, VALU-bound cast and
    # memory-bound MATERIAL overlap best three ways: -1 to -3 % at N = 1; with cost-balanced bands
    # three match two at N = 8, profiles/r06_rank_sim_partition.txt), two elsewhere (coffee +2-3 %
    # with three)
    args.streams_explicit = args.streams > 0   # (the configs[3] leg follows an explicit --streams)
    if args.streams <= 0:
        args.streams = 3 if args.config == "cornell" else 2
    args.pool = args.pool or scenes.default_pool(args.width, args.height, args.streams)
    # (the coffee scene without configs[2]'s multiscattering is its own workload)
    config_name = args.config + ("_noms" if args.config == "coffee" and args.no_multiscattering else "")
    filt = scene.filter_params()
    from directcomputeraytracing_amd.partition import halo_for_radius, render_rows
    halo = max(1, halo_for_radius(filt.radius, args.height))

    def make_tracer(pool, part, bands=None):
        t = WavefrontPathTracer(path_pool_size=pool, iterations_per_render=args.iterations, device=device)
        t.on_scene_loaded(scene)
        t.set_mode(args.mode)
        t.set_image_batch(args.image_batch)
        if bands is not None:
            t.set_film_bands(bands, halo)
        elif part is not None:
            t.set_film_partition(*part, halo)
        return t

    # cost-balanced film bands: the rays per film row of one probe image, the same
    # on every rank (exact, schedule-independent), cut into world x K contiguous equal-cost bands
    # dealt round-robin: pipeline s of rank r takes band s * world + r (make_pipelines), so a cost
    # trend down the image (time per ray is not uniform) evens out over the ranks. Not timed.
    K = max(1, args.streams)
    interleave = args.interleave == "on" or (args.interleave == "auto" and world > 1)
    B = max(1, args.bands_per_rank) if interleave else K      # bands per rank
    row_cost = None
    rank_bands = None
    if args.partition == "balanced" and world * B > 1 and args.mode == "wavefront":
        from directcomputeraytracing_amd import probe_row_cost
        from directcomputeraytracing_amd.partition import balanced_bands
        row_cost = probe_row_cost(scene, device=device)
        rank_bands = balanced_bands(row_cost, world * B, halo)[rank::world]

    # K concurrent pipelines per GPU (--streams), each on its own stream from its own host
    # thread. N = 1: pipeline s renders cost-balanced band s (disjoint film supports, summed on
    # the device by add_film_device). N > 1 (interleaved): the K pipelines share the rank's
    # bands and split the images; pipeline 0 convolves them all in image order.
    # (a pipeline's pool just short of a whole number of batches grows by <= 8 %: one drain less)
    def build_pipelines(cost):
        return make_pipelines(scene, args.pool, streams=K, images=args.steps * world, iterations=args.iterations,
                              world=world, rank=rank, stripe=args.stripe, mode=args.mode, image_batch=args.image_batch,
                              device=device, row_cost=cost, interleave=interleave, bands_per_rank=B)

    tracers = build_pipelines(row_cost)
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
        # the K pipelines' films into tracer 0's (disjoint supports: bit-exact sum); interleaved
        # pipelines already convolved into tracer 0's film
        if interleave:
            return
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
        for t in ([] if interleave else tracers[1:]):
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
    prepare_pipelines(tracers, images)     # sample textures of the timed batches + graph: not timed work
    snapshots = bool(args.snapshot_spp and args.snapshot_spp < images)

    calibration = None
    if dist is not None and row_cost is not None and args.calibrate > 0:
        # time per ray is not uniform over the film (deeper traversals lower in the Cornell
        # image), so the probe's ray counts leave the ranks a few % apart. Calibration rounds:
        # untimed renders of the timed workload (other seeds), the median rank times gathered, the
        # bands re-cut at equal time (partition.refine_row_cost -- every rank computes the same
        # cut from the same gathered times) and the pipelines rebuilt and prepared on it
        import torch
        from directcomputeraytracing_amd.partition import balanced_bands, refine_row_cost
        calibration = {"rounds": args.calibrate, "rank_ms_per_step": []}
        for _ in range(args.calibrate):
            runs_s = []
            for rep in range(3):                   # (the median of three: a single run is +-1.5 %)
                barrier_sync()
                t0 = time.perf_counter()
                render_all(20_000 + rep * images, images)
                for t in tracers:
                    t.synchronize()
                runs_s.append(time.perf_counter() - t0)
            mine = torch.tensor([float(np.median(runs_s))], dtype=torch.float64, device="cuda" if on_device else "cpu")
            gathered = [torch.zeros_like(mine) for _ in range(world)]
            dist.all_gather(gathered, mine)
            calib_s = [float(g.item()) for g in gathered]
            calibration["rank_ms_per_step"].append([round(x * 1e3 / args.steps, 3) for x in calib_s])
            all_bands = balanced_bands(row_cost, world * B, halo)
            row_cost = refine_row_cost(row_cost, [all_bands[r::world] for r in range(world)], calib_s, halo)
            rank_bands = balanced_bands(row_cost, world * B, halo)[rank::world]
            for t in tracers:
                t.destroy()
            tracers = build_pipelines(row_cost)
            tracer = tracers[0]
            for t in tracers:
                t.clear_film()
            if args.warmup:
                render_all(10_000, args.warmup)
            prepare_pipelines(tracers, images)

    def timed_run():
        """One timed repeat of exactly K steps: (wall s, this rank's render s, reduce s)."""
        for t in tracers:
            t.clear_film()
            t.reset_stats()
        barrier_sync()
        t0 = time.perf_counter()
        t_render = t_reduce = 0.0
        if snapshots:
            # progressive rendering (configs[4]): every K images the films so far are summed
            # over the pipelines and reduced onto rank 0 (a preview); the tracers' films keep
            # accumulating, so the last snapshot is the whole render
            done = 0
            while done < images:
                n = min(args.snapshot_spp, images - done)
                t1 = time.perf_counter()
                render_all(done, n)
                t2 = time.perf_counter()
                done += n
                snapshot_film()
                t_render += t2 - t1
                t_reduce += time.perf_counter() - t2
        else:
            render_all(0, images)
            combine_films()
            tracer.synchronize()
            t_render = time.perf_counter() - t0
            if dist is not None:
                t1 = time.perf_counter()
                reduce_film()
                if on_device:
                    import torch
                    torch.cuda.synchronize()
                t_reduce = time.perf_counter() - t1
        barrier_sync()
        return time.perf_counter() - t0, t_render, t_reduce

    runs = [timed_run() for _ in range(max(1, args.repeats))]
    rays = 0
    for t in tracers:
        c = t.counters()
        rays += c["extension_rays"] + c["shadow_rays"]
    walls = [r[0] for r in runs]
    rank_render = [r[1] for r in runs]
    rank_reduce = [r[2] for r in runs]
    per_rank = None
    if dist is not None:
        import torch
        assert dist.get_world_size() == args.gpus, f"--gpus {args.gpus} but the process group has {dist.get_world_size()} ranks"
        dev = "cuda" if on_device else "cpu"
        tw = torch.tensor(walls, dtype=torch.float64, device=dev)
        dist.all_reduce(tw, op=dist.ReduceOp.MAX)          # each repeat: the slowest rank's wall time
        walls = [float(x) for x in tw.cpu()]
        tr = torch.tensor([float(rays)], dtype=torch.float64, device=dev)
        dist.all_reduce(tr, op=dist.ReduceOp.SUM)
        rays = float(tr.item())
        mine = torch.tensor([float(np.median(rank_render)), float(np.median(rank_reduce))], dtype=torch.float64, device=dev)
        gathered = [torch.zeros_like(mine) for _ in range(world)]
        dist.all_gather(gathered, mine)
        per_rank = [[float(x) for x in g.cpu()] for g in gathered]
    elapsed = float(np.median(walls))

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
        tracer = make_tracer(args.pool, (world, rank, args.stripe) if world > 1 else None,
                             rank_bands if (rank_bands is not None and world > 1) else None)
    roof = cast_roofline(tracer, R, filt, {"config": config_name, "resolution": [args.width, args.height], "images": R,
                                           "path_pool": args.pool, "world": world}, args.traffic_json)
    st, cr, tm = roof.pop("_stats"), roof.pop("_counters"), roof.pop("_timing")
    pmc, pmc_src = roof.pop("_pmc")
    # whole-pipeline figure ("and for the whole pipeline"): the reference's
    # algorithmic bytes of every stage for the timed images (cast terms, CONTROL + MATERIAL
    # per path-iteration = per extension ray, NEW_PATH per new path, the film pass per pixel
    # x image), from the roofline leg's counts of the same images, over the timed region's
    # wall time, per GPU. These bytes are largely served from LDS / L2 / MALL: the figure is
    # an algorithmic rate, not an HBM measurement (the HBM statement is roofline.frac).
    film_bytes = FILM_BYTES_BASE + FILM_BYTES_PER_TAP * (2 * int(filt.radius + 0.5) + 1) ** 2
    pipe_bytes_R = (roof["bytes_per_launch"] * roof["launches"] + (CONTROL_BYTES + MATERIAL_BYTES) * cr["extension_rays"]
                    + NEW_PATH_BYTES * cr["new_paths"] + film_bytes * args.width * args.height * R / world)
    pipe_achieved = pipe_bytes_R * (images / R) / elapsed / 1e9

    result = {
        "metric": ("Mrays/s and ms/spp at 1920x1080, 8-bounce wavefront" if args.config == "cornell"
                   else f"Mrays/s and ms/spp at {args.width}x{args.height}, {config_name} config, wavefront"),
        "value": round(rays / elapsed / 1e6, 2),
        "unit": "Mrays/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(elapsed * 1e3 / args.steps, 3),
        "ms_per_spp": round(elapsed * 1e3 / images, 3),
        "repeats": len(walls),
        "repeat_ms_per_spp": [round(w * 1e3 / images, 3) for w in walls],
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "f32",
        "data": "synthetic",
        "config": {"workload": workload.format(spp=images), "name": config_name,
                   "resolution": [args.width, args.height], "spp": images,
                   "max_bounce": args.bounces if args.config == "cornell" else scene.frame_params(0).max_bounce_count,
                   "path_pool": args.pool, "streams_per_gpu": K, "snapshot_spp": args.snapshot_spp or images,
                   "parallelism": (f"film {'cost-balanced bands' if rank_bands is not None else 'stripes'} x{world}"
                                   if world > 1 else "single GPU")
                                  + (f", {K} concurrent pipelines per GPU" if K > 1 else "")
                                  + (f" (image-interleaved over the rank's {B} band(s))" if interleave and K > 1 else "")
                                  + (" (cost-balanced bands)" if rank_bands is not None and world == 1 else ""),
                   "partition": args.partition if rank_bands is not None else ("stripes" if world * K > 1 else "none"),
                   "interleave": interleave, "bands_per_rank": B if rank_bands is not None else None,
                   "rays": int(rays)},
        "roofline": roof,
        "pipeline_roofline": pipeline_roofline(pmc, pmc_src, images / world / elapsed, pipe_achieved, pipe_bytes_R / R),
        "material": material_roofline(tm, pmc, pmc_src),
        "cpu_baseline": None,
    }
    if per_rank is not None:
        # diagnosable first 8-GPU run: every rank's render time (its stripes + halo rows) and the
        # RCCL film reduce, medians over the repeats; the halo overhead is rows rendered / owned
        if rank_bands is not None:
            from directcomputeraytracing_amd.partition import band_render_rows
            owned = sum(b - a for a, b in rank_bands)
            rendered = sum(len(band_render_rows(args.height, [b], halo)) for b in rank_bands)
        else:
            owned = len(render_rows(args.height, world, rank, args.stripe, 0))
            rendered = len(render_rows(args.height, world, rank, args.stripe, halo))
        result["multi_gpu"] = {"world_size": world, "per_rank_render_ms": [round(r[0] * 1e3, 3) for r in per_rank],
                               "per_rank_reduce_ms": [round(r[1] * 1e3, 3) for r in per_rank],
                               "reduce": "torch.distributed.reduce(SUM) of the RGBA32F film, "
                                         + ("RCCL over xGMI" if on_device else args.dist_backend),
                               "film_bytes": args.width * args.height * 16,
                               "rank0_rows_owned": owned, "rank0_rows_rendered": rendered,
                               "rank0_halo_overhead": round(rendered / max(1, owned) - 1.0, 4),
                               "calibration": calibration}
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        label = "1920x1080 8-bounce Cornell" if args.config == "cornell" else f"{args.config} config"
        result["cpu_baseline"] = cpu_baseline(scene, luts_arrays, args.cpu_seconds, label)
    tracer.destroy()
    if rank == 0 and world == 1 and args.config == "cornell" and args.spaceship_spp > 0 and args.mode == "wavefront":
        result["spaceship"] = spaceship_leg(args, luts_arrays)
    if rank == 0:
        print(json.dumps(result), flush=True)
    if dist is not None:
        dist.destroy_process_group()


def cast_roofline(tracer, R, filt, workload_key, traffic_json=None) -> dict:
    """The merged EXTENSION+SHADOW cast launch over images 0..R-1 of the tracer's scene:
    algorithmic bytes (the reference's traversal counts x SURVEY 8(d) bytes per unit, from
    the instrumented variant), HIP-event launch time, and the HBM bytes a committed
    rocprofv3 PMC profile of THIS workload measured per launch (tools/prof_config.sh /
    tools/profile.sh + tools/pmc_traffic.py)."""
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
    info = tracer.info()
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
    alg = bytes_per_launch / (avg_ms * 1e-3) / 1e9
    pmc, pmc_src = find_pmc_profile(workload_key, traffic_json)
    traffic, traffic_src, valu = None, "no committed PMC profile of this workload", None
    if pmc is not None and pmc.get("ext_hbm_bytes_per_launch"):
        traffic = pmc["ext_hbm_bytes_per_launch"]
        traffic_src = f"{pmc_src}: rocprofv3 PMC, FETCH_SIZE x2 + WRITE_SIZE per cast launch, same workload"
        if pmc.get("ext_valu_issue_frac"):
            # what the launch does bound: the VALU issue slots (a wave64 instruction takes 2
            # cycles of its SIMD) used over the launch's active cycles, the tail included
            valu = {"valu_issue_frac": round(pmc["ext_valu_issue_frac"], 4),
                    "valu_insts_per_launch": pmc.get("ext_valu_insts_per_launch"),
                    "implied_clock_ghz": None if pmc.get("ext_implied_clock_ghz") is None else round(pmc["ext_implied_clock_ghz"], 3),
                    "basis": "SQ_INSTS_VALU x 2 cycles / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) per cast launch, "
                             "same PMC profile"}
    hbm = None if traffic is None else traffic / (avg_ms * 1e-3) / 1e9
    # what bounds the launch, from the evidence: a scene resident in the LDS scene cache
    # (Cornell) runs node / triangle fetches from LDS and is VALU-issue bound;
    # a scene that does not fit walks its nodes through L2 / MALL (L2-miss latency bound)
    bound = "lds/valu (scene in the LDS cache)" if info["scene_in_lds"] else "memory latency (L2/MALL-resident scene)"
    return {"bound": bound,
            "kernel": "cast_kernel (EXTENSION_RAY_CAST + SHADOW_RAY_CAST, one launch)" if merged
                      else "extension_kernel (EXTENSION_RAY_CAST)",
            "achieved": None if hbm is None else round(hbm, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
            "frac": None if hbm is None else round(hbm / HBM_PEAK_GBS, 4),
            "basis": "measured HBM: rocprofv3 PMC bytes per cast launch (traffic) / HIP-event launch time",
            "traffic": traffic, "traffic_source": traffic_src,
            "compute": valu,
            "achieved_algorithmic": round(alg, 1), "frac_algorithmic": round(alg / HBM_PEAK_GBS, 4),
            "algorithmic_basis": "the reference's traversal counts (node visits, triangle tests, BLAS entries, "
                                 "from the instrumented kernel) x SURVEY 8(d)'s bytes per unit, wherever the bytes "
                                 "are served from (LDS scene cache, L1, L2, MALL or HBM)",
            "bytes_per_launch": int(bytes_per_launch), "avg_launch_us": round(avg_ms * 1e3, 2),
            "launches": int(launches), "images": R, "scene_in_lds": bool(info["scene_in_lds"]),
            "launch": {k: int(info[k]) for k in ("cast_grid", "cast_block", "cached_nodes", "cached_triangles", "traversal_stack",
                                                 "pair_traversal", "material_grid", "material_lds", "cast_identity",
                                                 "stack_lds_rows", "ring_rows", "cast_waves_per_cu")},
            "extension_rays": int(cr["extension_rays"]), "shadow_rays": int(cr["shadow_rays"]),
            "per_ext_ray": {"nodes": st["ext_node_visits"] / max(1, cr["extension_rays"]),
                            "tris": st["ext_triangle_tests"] / max(1, cr["extension_rays"]),
                            "blas": st["ext_blas_entries"] / max(1, cr["extension_rays"])},
            "per_shadow_ray": {"nodes": st["shadow_node_visits"] / max(1, cr["shadow_rays"]),
                               "tris": st["shadow_triangle_tests"] / max(1, cr["shadow_rays"]),
                               "blas": st["shadow_blas_entries"] / max(1, cr["shadow_rays"])},
            "_stats": st, "_counters": cr, "_timing": tm, "_pmc": (pmc, pmc_src)}


def pipeline_roofline(pmc, pmc_src, images_per_s, alg_achieved, alg_bytes_per_image) -> dict:
    """The whole pipeline on one GPU ("and for the whole pipeline"): the HBM bytes
    per image that the committed PMC profile of this workload measured over every per-image
    kernel (tools/pmc_traffic.py pipeline_hbm_bytes_per_image: cast, MATERIAL, CONTROL, film,
    image sequencing), times the images this GPU renders per second in the timed region. The
    reference's algorithmic bytes (largely served from LDS / L2 / MALL, so above the HBM peak
    on cache-resident scenes) stay beside it as achieved_algorithmic."""
    out = {"peak": HBM_PEAK_GBS, "unit": "GB/s", "achieved": None, "frac": None, "traffic": None}
    if alg_achieved is not None:
        out.update(achieved_algorithmic=round(alg_achieved, 1), frac_algorithmic=round(alg_achieved / HBM_PEAK_GBS, 4),
                   bytes_per_spp_algorithmic=int(alg_bytes_per_image),
                   algorithmic_basis="per GPU: algorithmic bytes of cast + CONTROL (92 B) + MATERIAL (600 B) per "
                                     "path-iteration + NEW_PATH (88 B) per new path + film pass per pixel-image (SURVEY "
                                     "8(d)) over the timed region's wall time; mostly LDS / cache served")
    if pmc is None or not pmc.get("pipeline_hbm_bytes_per_image"):
        out["bound"] = "unmeasured (no committed PMC profile of this workload)"
        return out
    t = pmc["pipeline_hbm_bytes_per_image"]
    achieved = t * images_per_s / 1e9
    out.update(bound="measured HBM", achieved=round(achieved, 1), frac=round(achieved / HBM_PEAK_GBS, 4), traffic=t,
               traffic_by_kernel={k: int(v) for k, v in sorted(pmc.get("pipeline_hbm_bytes_per_image_by_kernel", {}).items())},
               basis="rocprofv3 PMC HBM bytes per image summed over every per-image kernel (FETCH_SIZE x2 + WRITE_SIZE) "
                     "x the images this GPU rendered per second of the timed region",
               traffic_source=f"{pmc_src}: pipeline_hbm_bytes_per_image")
    return out


def find_pmc_profile(workload_key, traffic_json=None):
    """The newest committed tools/pmc_traffic.py summary (profiles/r*_pmc_traffic*.json) whose
    recorded workload is this run's: (dict, path) or (None, None)."""
    cands = [Path(traffic_json)] if traffic_json else sorted((ROOT / "profiles").glob("r*_pmc_traffic*.json"), reverse=True)
    for tj in cands:
        try:
            d = json.loads(tj.read_text())
        except Exception:
            continue
        if d.get("workload") == workload_key and d.get("ext_hbm_bytes_per_launch"):
            return d, str(tj.relative_to(ROOT) if tj.is_relative_to(ROOT) else tj)
    return None, None


def material_roofline(tm, pmc, pmc_src) -> dict:
    """MATERIAL's own statement: the PMC-measured HBM bytes per launch of the same workload over
    its average HIP-event launch time (the roofline leg's timed launches), plus VALU issue."""
    launches = tm.get("material_launches", 0)
    avg_ms = tm["material_kernel_ms"] / launches if launches else None
    out = {"kernel": "material_kernel (MATERIAL)", "avg_launch_us": None if avg_ms is None else round(avg_ms * 1e3, 2),
           "launches": int(launches), "peak": HBM_PEAK_GBS, "unit": "GB/s", "achieved": None, "frac": None,
           "traffic": None, "compute": None}
    if pmc is None or not pmc.get("material_hbm_bytes_per_launch") or avg_ms is None:
        out["traffic_source"] = "no committed PMC profile of this workload"
        return out
    b = pmc["material_hbm_bytes_per_launch"]
    achieved = b / (avg_ms * 1e-3) / 1e9
    out.update(achieved=round(achieved, 1), frac=round(achieved / HBM_PEAK_GBS, 4), traffic=b,
               read_bytes=pmc.get("material_read_bytes_per_launch"), write_bytes=pmc.get("material_write_bytes_per_launch"),
               traffic_source=f"{pmc_src}: rocprofv3 PMC, FETCH_SIZE x2 + WRITE_SIZE per MATERIAL launch, same workload",
               bound="memory latency (dependent hit -> triangle -> material fetches; DESIGN section 4)")
    if pmc.get("material_valu_issue_frac"):
        out["compute"] = {"valu_issue_frac": round(pmc["material_valu_issue_frac"], 4),
                          "basis": "SQ_INSTS_VALU x 2 cycles / (GRBM_GUI_ACTIVE / 8 XCDs x 1024 SIMDs) per MATERIAL launch"}
    return out


def spaceship_leg(args, luts_arrays) -> dict:
    """configs[3] on this GPU (the traversal that touches HBM: 2 x 261 k-triangle hull BLAS
    instanced 8 times, 3840x2160, 8 bounces): ms/spp over a few images (median of the
    repeats, two concurrent pipelines as in the headline), then the cast roofline of the
    same images on one pipeline with the HBM fraction from its committed PMC profile."""
    from directcomputeraytracing_amd import Scene, WavefrontPathTracer, render_images_concurrently, scenes
    from directcomputeraytracing_amd.partition import halo_for_radius, stream_partition
    scene = Scene((3840, 2160))
    desc = scenes.setup_config(scene, "spaceship", args.scene_dir)
    W, H = scene.resolution
    # two pipelines unless --streams was given (the headline's automatic count is Cornell's)
    K = args.streams if getattr(args, "streams_explicit", False) else 2
    pool = scenes.default_pool(W, H, K)
    filt = scene.filter_params()
    halo = max(1, halo_for_radius(filt.radius, H))
    n = args.spaceship_spp
    subs = []
    try:
        for s_ in range(K):
            t = WavefrontPathTracer(path_pool_size=pool // K, iterations_per_render=args.iterations)
            t.on_scene_loaded(scene)
            if K > 1:
                t.set_film_partition(*stream_partition(H, 1, 0, K, s_, args.stripe), halo)
            subs.append(t)
        for t in subs:
            t.clear_film()
        render_images_concurrently(subs, 10_000, 1, filt)      # warm-up (graphs)
        for t in subs:
            t.prepare_images(n)
        walls = []
        for _ in range(max(1, min(args.repeats, 3))):
            for t in subs:
                t.clear_film()
                t.reset_stats()
            t0 = time.perf_counter()
            render_images_concurrently(subs, 0, n, filt)
            walls.append(time.perf_counter() - t0)
        rays = sum(t.counters()["extension_rays"] + t.counters()["shadow_rays"] for t in subs)
    finally:
        for t in subs:
            t.destroy()
    el = float(np.median(walls))
    tr = WavefrontPathTracer(path_pool_size=pool, iterations_per_render=args.iterations)
    try:
        tr.on_scene_loaded(scene)
        roof = cast_roofline(tr, n, filt, {"config": "spaceship", "resolution": [W, H], "images": n,
                                           "path_pool": pool, "world": 1})
    finally:
        tr.destroy()
    tm = roof.pop("_timing")
    pmc, pmc_src = roof.pop("_pmc")
    roof.pop("_stats"), roof.pop("_counters")
    return {"workload": f"{desc}, {n} spp, 1 GPU, {K} concurrent pipelines", "ms_per_spp": round(el * 1e3 / n, 3),
            "repeat_ms_per_spp": [round(w * 1e3 / n, 3) for w in walls], "mrays_per_s": round(rays / el / 1e6, 2),
            "path_pool": pool, "roofline": roof, "material": material_roofline(tm, pmc, pmc_src),
            "pipeline_roofline": pipeline_roofline(pmc, pmc_src, n / el, None, None)}


if __name__ == "__main__":
    main()
