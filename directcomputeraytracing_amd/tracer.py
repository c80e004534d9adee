"""``CWavefrontPathTracer`` (Source/WavefrontPathTracer.h:7-101) on MI355X.

A thin host mirror over the C ABI: every call goes to ``libdcrt.so`` (gfx950
kernels). Method names follow the reference's ``CPathTracer`` interface
(Source/PathTracer.h:3-31): ``create``/``destroy``/``on_scene_loaded``/
``render``/``reset_image``/``is_image_complete``/``acquire_film_clear_trigger``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _abi
from ._abi import check
from .scene import Scene

RAY_DTYPE = np.dtype([("origin", "<f4", 3), ("t_max", "<f4"), ("direction", "<f4", 3), ("t_min", "<f4")])
HIT_DTYPE = np.dtype([("t", "<f4"), ("u", "<f4"), ("v", "<f4"), ("triangle_id", "<u4"), ("instance_index", "<u4")])
assert RAY_DTYPE.itemsize == 32 and HIT_DTYPE.itemsize == 20

MATH_SIN, MATH_COS, MATH_EXP, MATH_ATAN = range(4)


def make_rays(origins, directions, t_min=0.0, t_max=np.inf) -> np.ndarray:
    o = np.asarray(origins, np.float32).reshape(-1, 3)
    d = np.asarray(directions, np.float32).reshape(-1, 3)
    r = np.zeros(len(o), RAY_DTYPE)
    r["origin"], r["direction"] = o, d
    r["t_min"], r["t_max"] = t_min, t_max
    return r


class WavefrontPathTracer:
    """CWavefrontPathTracer: path pool, queues and kernels resident in HBM."""

    def __init__(self, path_pool_size: int = 0, iterations_per_render: int = 0, device: int = 0,
                 stream: int | None = None, debug_rng: bool = False):
        self._lib = _abi.load_library()
        self._h = None
        self.create(path_pool_size, iterations_per_render, device, stream, debug_rng)

    # ---- CPathTracer --------------------------------------------------------
    def create(self, path_pool_size=0, iterations_per_render=0, device=0, stream=None, debug_rng=False):
        cfg = _abi.TracerConfig(int(path_pool_size), int(iterations_per_render), int(device),
                                C.c_void_p(stream or 0), 1 if debug_rng else 0)
        h = C.c_void_p()
        check(self._lib.dcrt_tracer_create(C.byref(cfg), C.byref(h)), "Create")
        self._h = h
        self.width = self.height = 0
        self.filter = _abi.FilterParams(_abi.FILTER_BOX, 1.0, 1.5, 1 / 3, 1 / 3, 3)

    def destroy(self):
        if self._h:
            self._lib.dcrt_tracer_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.destroy()
        except Exception:
            pass

    def on_scene_loaded(self, scene: Scene, frame_seed: int = 0) -> None:
        """Upload the flattened scene and the camera/film constants (OnSceneLoaded)."""
        flat = scene.flat()
        check(self._lib.dcrt_tracer_upload_scene(self._h, C.byref(flat)), "OnSceneLoaded")
        self.set_frame_params(scene.frame_params(frame_seed))
        self.filter = scene.filter_params()

    def set_frame_params(self, params: _abi.FrameParams) -> None:
        check(self._lib.dcrt_tracer_set_frame_params(self._h, C.byref(params)), "SetFrameParams")
        self.width, self.height = params.resolution[0], params.resolution[1]

    def set_film_partition(self, world_size: int, rank: int, stripe_height: int = 64, halo_rows: int = 0) -> None:
        p = _abi.FilmPartition(world_size, rank, stripe_height, halo_rows)
        check(self._lib.dcrt_tracer_set_film_partition(self._h, C.byref(p)), "SetFilmPartition")

    def set_film_bands(self, bands, halo_rows: int = 0) -> None:
        """Own the rows of the (y0, y1) bands (ascending, disjoint), path-trace them plus halo_rows
        beyond each and convolve only them (dcrt_tracer_set_film_bands)."""
        flat = np.asarray([y for b in bands for y in b], np.uint32)
        check(self._lib.dcrt_tracer_set_film_bands(self._h, flat.ctypes.data_as(C.POINTER(C.c_uint32)), len(bands),
                                                   int(halo_rows)), "SetFilmBands")

    def set_row_cost_probe(self, enable: bool) -> None:
        """Count the rays cast per film row from now on (cleared when turned on)."""
        check(self._lib.dcrt_tracer_set_row_cost_probe(self._h, 1 if enable else 0), "SetRowCostProbe")

    def read_row_cost(self) -> np.ndarray:
        out = np.empty(self.height, np.uint32)
        check(self._lib.dcrt_tracer_read_row_cost(self._h, out.ctypes.data_as(C.POINTER(C.c_uint32))), "ReadRowCost")
        return out

    def render(self, max_iterations: int = 0) -> None:
        check(self._lib.dcrt_tracer_render(self._h, int(max_iterations)), "Render")

    def render_images(self, first_seed: int, count: int, filter_params: _abi.FilterParams | None = None,
                      seed_stride: int = 1, convolve: bool = True) -> None:
        """Images first_seed + k * seed_stride, k < count; convolve=False keeps every image's
        samples (slot k) for accumulate_images instead of running the film pass."""
        f = filter_params or self.filter
        if seed_stride == 1 and convolve:
            check(self._lib.dcrt_tracer_render_images(self._h, int(first_seed), int(count), C.byref(f)), "RenderImages")
        else:
            check(self._lib.dcrt_tracer_render_images_strided(self._h, int(first_seed), int(seed_stride), int(count),
                                                              1 if convolve else 0, C.byref(f)), "RenderImagesStrided")

    def image_sample_ptrs(self, image: int) -> tuple[int, int]:
        pos, val = C.c_void_p(), C.c_void_p()
        check(self._lib.dcrt_tracer_image_sample_ptrs(self._h, int(image), C.byref(pos), C.byref(val)), "ImageSamplePtrs")
        return pos.value or 0, val.value or 0

    def accumulate_images(self, positions, values, filter_params: _abi.FilterParams | None = None) -> None:
        """SampleConvolution of the images whose sample textures sit at these device pointers, in order."""
        f = filter_params or self.filter
        n = len(positions)
        P = (C.c_void_p * max(1, n))(*positions)
        V = (C.c_void_p * max(1, n))(*values)
        check(self._lib.dcrt_tracer_accumulate_images(self._h, P, V, n, C.byref(f)), "AccumulateImages")

    def prepare_images(self, count: int) -> None:
        """Allocate / capture what render_images(count) would on its first call."""
        check(self._lib.dcrt_tracer_prepare_images(self._h, int(count)), "PrepareImages")

    def set_image_batch(self, images: int = 0) -> None:
        """Images per render_images batch (0 = automatic)."""
        check(self._lib.dcrt_tracer_set_image_batch(self._h, int(images)), "SetImageBatch")

    def set_mode(self, mode: str) -> None:
        """"wavefront" (CWavefrontPathTracer) or "megakernel" (CMegakernelPathTracer) for render_images."""
        check(self._lib.dcrt_tracer_set_mode(self._h, {"wavefront": 0, "megakernel": 1}[mode]), "SetMode")

    def reset_image(self) -> None:
        check(self._lib.dcrt_tracer_reset_image(self._h), "ResetImage")

    def is_image_complete(self) -> bool:
        v = C.c_int()
        check(self._lib.dcrt_tracer_is_image_complete(self._h, C.byref(v)), "IsImageComplete")
        return bool(v.value)

    def acquire_film_clear_trigger(self) -> bool:
        v = C.c_int()
        check(self._lib.dcrt_tracer_acquire_film_clear_trigger(self._h, C.byref(v)), "AcquireFilmClearTrigger")
        return bool(v.value)

    # ---- film --------------------------------------------------------------
    def clear_film(self) -> None:
        check(self._lib.dcrt_tracer_clear_film(self._h), "ClearFilm")

    def accumulate_film(self, filter_params: _abi.FilterParams | None = None) -> None:
        f = filter_params or self.filter
        check(self._lib.dcrt_tracer_accumulate_film(self._h, C.byref(f)), "SampleConvolution")

    def read_film(self) -> np.ndarray:
        out = np.empty((self.height, self.width, 4), np.float32)
        check(self._lib.dcrt_tracer_read_film(self._h, out.ctypes.data_as(_abi._FP)), "ReadFilm")
        return out

    def read_samples(self):
        pos = np.empty((self.height, self.width, 2), np.float32)
        val = np.empty((self.height, self.width, 4), np.float32)
        check(self._lib.dcrt_tracer_read_samples(self._h, pos.ctypes.data_as(_abi._FP), val.ctypes.data_as(_abi._FP)),
              "ReadSamples")
        return pos, val

    def read_rng(self) -> np.ndarray:
        out = np.empty((self.height, self.width, 4), np.uint32)
        check(self._lib.dcrt_tracer_read_rng(self._h, out.ctypes.data_as(C.POINTER(C.c_uint32))), "ReadRng")
        return out

    def film_device_ptr(self) -> int:
        p = C.c_void_p()
        check(self._lib.dcrt_tracer_film_device_ptr(self._h, C.byref(p)), "FilmDevicePtr")
        return p.value or 0

    def sample_device_ptrs(self) -> tuple[int, int]:
        """Device pointers of the current image's sample textures (R32G32F positions, RGBA32F
        values): what the reference's SampleConvolution pass reads."""
        pos, val = C.c_void_p(), C.c_void_p()
        check(self._lib.dcrt_tracer_sample_device_ptrs(self._h, C.byref(pos), C.byref(val)), "SampleDevicePtrs")
        return pos.value or 0, val.value or 0

    def copy_film_device(self, d_dst: int) -> None:
        check(self._lib.dcrt_tracer_copy_film_device(self._h, C.c_void_p(d_dst)), "CopyFilmDevice")

    def add_film_device(self, d_src: int) -> None:
        """film += the RGBA32F film at device address d_src (another partition's film)."""
        check(self._lib.dcrt_tracer_add_film_device(self._h, C.c_void_p(d_src)), "AddFilmDevice")

    def resolve_image(self, params: _abi.PostFxParams | None = None, with_luminance: bool = False):
        """Post-processing (exposure + Reinhard) into sRGB8 RGBA, H x W x 4 uint8."""
        p = params or _abi.PostFxParams(1, 1, 15.0, 1.0)
        out = np.empty((self.height, self.width, 4), np.uint8)
        lum = C.c_float()
        check(self._lib.dcrt_tracer_resolve_image(self._h, C.byref(p), out.ctypes.data_as(C.POINTER(C.c_uint8)),
                                                  C.byref(lum)), "ResolveImage")
        return (out, lum.value) if with_luminance else out

    # ---- statistics ----------------------------------------------------------
    def counters(self) -> dict:
        s = _abi.RayStats()
        check(self._lib.dcrt_tracer_counters(self._h, C.byref(s)), "Counters")
        return {k: getattr(s, k) for k, _ in _abi.RayStats._fields_}

    def set_instrumentation(self, counters: bool, ext_timing: bool) -> None:
        check(self._lib.dcrt_tracer_set_instrumentation(self._h, int(counters), int(ext_timing)), "SetInstrumentation")

    def traversal_stats(self) -> dict:
        s = _abi.TraversalStats()
        check(self._lib.dcrt_tracer_traversal_stats(self._h, C.byref(s)), "TraversalStats")
        return {k: getattr(s, k) for k, _ in _abi.TraversalStats._fields_}

    def info(self) -> dict:
        """What the tracer chose for the uploaded scene (pool, LDS scene cache, variants)."""
        s = _abi.TracerInfo()
        check(self._lib.dcrt_tracer_get_info(self._h, C.byref(s)), "GetInfo")
        return {k: getattr(s, k) for k, _ in _abi.TracerInfo._fields_}

    def ring_spills(self) -> int:
        """Stack entries the spilling-stack cast kernel moved to its global columns (test hook)."""
        n = C.c_uint64(0)
        check(self._lib.dcrt_tracer_debug_ring_spills(self._h, C.byref(n)), "DebugRingSpills")
        return int(n.value)

    def reset_stats(self) -> None:
        check(self._lib.dcrt_tracer_reset_stats(self._h), "ResetStats")

    def synchronize(self) -> None:
        check(self._lib.dcrt_tracer_synchronize(self._h), "Synchronize")

    def luts(self) -> _abi.BxDFLuts:
        l = _abi.BxDFLuts()
        check(self._lib.dcrt_tracer_get_luts(self._h, C.byref(l)), "GetLuts")
        return l

    def set_luts(self, luts: _abi.BxDFLuts) -> None:
        check(self._lib.dcrt_tracer_set_luts(self._h, C.byref(luts)), "SetLuts")

    # ---- kernel-level entry points -------------------------------------------
    def trace_rays(self, rays: np.ndarray, features: int = _abi.FEATURE_DEFAULT) -> np.ndarray:
        rays = np.ascontiguousarray(rays, RAY_DTYPE)
        hits = np.zeros(len(rays), HIT_DTYPE)
        check(self._lib.dcrt_tracer_trace_rays(self._h, rays.ctypes.data_as(C.POINTER(_abi.Ray)), len(rays),
                                               hits.ctypes.data_as(C.POINTER(_abi.RayHit)), int(features)), "TraceRays")
        return hits

    def occluded(self, rays: np.ndarray, features: int = _abi.FEATURE_DEFAULT) -> np.ndarray:
        rays = np.ascontiguousarray(rays, RAY_DTYPE)
        out = np.zeros(len(rays), np.uint32)
        check(self._lib.dcrt_tracer_occluded(self._h, rays.ctypes.data_as(C.POINTER(_abi.Ray)), len(rays),
                                             out.ctypes.data_as(C.POINTER(C.c_uint32)), int(features)), "Occluded")
        return out

    def trace_rays_device(self, d_rays: int, count: int, d_hits: int, features: int = _abi.FEATURE_DEFAULT) -> None:
        check(self._lib.dcrt_tracer_trace_rays_device(self._h, C.c_void_p(d_rays), int(count), C.c_void_p(d_hits),
                                                      int(features)), "TraceRaysDevice")

    def math_eval(self, function: int, x: np.ndarray) -> np.ndarray:
        x = np.ascontiguousarray(x, np.float32)
        y = np.empty_like(x)
        check(self._lib.dcrt_device_math_eval(self._h, int(function), x.ctypes.data_as(_abi._FP), x.size,
                                              y.ctypes.data_as(_abi._FP)), "MathEval")
        return y


def srgb_thresholds() -> np.ndarray:
    out = np.empty(255, np.float32)
    check(_abi.load_library().dcrt_srgb_encode_thresholds(out.ctypes.data_as(_abi._FP)), "SrgbThresholds")
    return out


def save_bmp(path, rgba8: np.ndarray) -> None:
    """24-bit BMP (SaveImageToFile.cpp:92-182)."""
    a = np.ascontiguousarray(rgba8, np.uint8)
    h, w = a.shape[:2]
    check(_abi.load_library().dcrt_write_bmp(str(path).encode(), w, h, a.ctypes.data_as(C.POINTER(C.c_uint8))), "WriteBmp")


def device_count() -> int:
    lib = _abi.load_library()
    n = C.c_int()
    check(lib.dcrt_device_count(C.byref(n)))
    return n.value


def make_pipelines(scene, pool: int, streams: int = 2, images: int = 1, iterations: int = 16, world: int = 1,
                   rank: int = 0, stripe: int = 64, mode: str = "wavefront", image_batch: int = 0, device: int = 0,
                   debug_rng: bool = False, row_cost=None, fixed_pool: bool = False, interleave: bool = False,
                   bands_per_rank: int = 0) -> list:
    """The concurrent wavefront pipelines bench.py renders with, each a tracer with its share of
    `pool` slots (grown to whole batches of `images` images, partition.pipeline_pool), the
    filter's halo rows, its own stream. With `row_cost` (rays per film row, probe_row_cost) the
    film is cut into world x streams contiguous equal-cost bands (partition.balanced_bands) and
    pipeline s of rank r takes band s * world + r -- dealt round-robin, so every rank holds one
    band of each 1/streams of the film and a cost trend down the image evens out; without it, one GPU splits the film into
    `streams` equal horizontal bands and N GPUs deal this rank's round-robin stripes to its
    pipelines (partition.stream_partition). Their films have disjoint supports: add_film_device
    sums them into the rank's film bit for bit."""
    from .partition import balanced_bands, band_render_rows, halo_for_radius, pipeline_pool, render_rows, stream_partition
    W, H = scene.resolution
    halo = max(1, halo_for_radius(scene.filter_params().radius, H))
    K = max(1, streams)
    if interleave:
        return _make_interleaved(scene, pool, K, images, iterations, world, rank, stripe, mode, image_batch, device, debug_rng,
                                 row_cost, fixed_pool, bands_per_rank or K, halo)
    bands = balanced_bands(row_cost, world * K, halo) if row_cost is not None and world * K > 1 else None
    tracers = []
    try:
        for s_ in range(K):
            part = stream_partition(H, world, rank, K, s_, stripe) if (K > 1 or world > 1) and bands is None else None
            band = [bands[s_ * world + rank]] if bands is not None else None
            rows = (len(band_render_rows(H, band, halo)) if band is not None
                    else len(render_rows(H, *part, halo)) if part is not None else H)
            p = pipeline_pool(pool // K, rows, W, images) if not (image_batch or fixed_pool) else pool // K
            t = WavefrontPathTracer(path_pool_size=p, iterations_per_render=iterations, device=device, debug_rng=debug_rng)
            tracers.append(t)
            t.on_scene_loaded(scene)
            t.set_mode(mode)
            t.set_image_batch(image_batch)
            if band is not None:
                t.set_film_bands(band, halo)
            elif part is not None:
                t.set_film_partition(*part, halo)
    except BaseException:
        for t in tracers:
            t.destroy()
        raise
    return tracers


def _make_interleaved(scene, pool, K, images, iterations, world, rank, stripe, mode, image_batch, device, debug_rng, row_cost,
                      fixed_pool, bands_per_rank, halo) -> list:
    """make_pipelines(interleave=True): K tracers over the SAME rows -- the whole film on one GPU,
    the rank's share of it on N (`bands_per_rank` cost-balanced bands dealt round-robin, or the
    round-robin stripes without a row cost) -- that split the images instead of the rows
    (render_images_concurrently deals image j to pipeline j mod K). No halo rows between the
    pipelines of one GPU, and the pipelines carry statistically equal work."""
    from .partition import balanced_bands, band_render_rows, pipeline_pool, render_rows
    W, H = scene.resolution
    bands = part = None
    if world > 1:
        if row_cost is not None:
            B = max(1, bands_per_rank)
            bands = balanced_bands(row_cost, world * B, halo)[rank::world]
        else:
            part = (world, rank, stripe)
    rows = (len(band_render_rows(H, bands, halo)) if bands is not None
            else len(render_rows(H, *part, halo)) if part is not None else H)
    per = -(-images // K)
    px = max(1, -(-rows // 8) * 8 * -(-W // 8) * 8)
    p = pipeline_pool(pool // K, rows, W, per) if not (image_batch or fixed_pool) else pool // K
    tracers = []
    try:
        for _ in range(K):
            t = WavefrontPathTracer(path_pool_size=p, iterations_per_render=iterations, device=device, debug_rng=debug_rng)
            tracers.append(t)
            t.on_scene_loaded(scene)
            t.set_mode(mode)
            t.set_image_batch(image_batch)
            if bands is not None:
                t.set_film_bands(bands, halo)
            elif part is not None:
                t.set_film_partition(*part, halo)
            t.interleaved = True
            t.pool_images = max(1, p // px)
            t.rank_bands = bands
    except BaseException:
        for t in tracers:
            t.destroy()
        raise
    return tracers


def _run_threads(tracers, fn) -> None:
    """fn(index, tracer) on every tracer at once (one host thread each; the C ABI runs with the
    GIL released and every tracer owns its stream). An error in any tracer is raised here,
    after every thread has finished."""
    import threading
    errors = []

    def run(i, t):
        try:
            fn(i, t)
        except BaseException as e:   # re-raised in the caller's thread
            errors.append(e)

    if len(tracers) == 1:
        run(0, tracers[0])
    else:
        th = [threading.Thread(target=run, args=(i, t)) for i, t in enumerate(tracers)]
        for x in th:
            x.start()
        for x in th:
            x.join()
    if errors:
        raise errors[0]


def render_images_concurrently(tracers, first_seed: int, count: int, filter_params=None) -> None:
    """render_images on several tracers at once, then synchronize them all. Pipelines built
    with interleaved images (make_pipelines(interleave=True)) share their rows: tracer s renders
    images s, s + K, ... of each chunk without the film pass, and tracer 0 then convolves the
    chunk's images in image order from all K pipelines' sample textures (accumulate_images), so
    its film is the one-pipeline film bit for bit and the others' stay empty."""
    K = len(tracers)
    if K > 1 and getattr(tracers[0], "interleaved", False):
        # chunks the pipelines' pools hold whole (one batch each, with its virtual start)
        chunk = K * max(1, min(getattr(t, "pool_images", 1) for t in tracers))
        for c0 in range(0, count, chunk):
            n = min(chunk, count - c0)
            _run_threads(tracers, lambda s, t: t.render_images(first_seed + c0 + s, len(range(s, n, K)), filter_params,
                                                               seed_stride=K, convolve=False) if s < n else None)
            for t in tracers:
                t.synchronize()
            # image k of a pipeline's call sits in its sample slot k: slot 0's pointers plus k
            # whole-film strides (one ABI call per pipeline, not one per image)
            W, H = tracers[0].width, tracers[0].height
            base = [t.image_sample_ptrs(0) for t in tracers[:min(K, n)]]
            pos = [base[j % K][0] + (j // K) * W * H * 8 for j in range(n)]
            val = [base[j % K][1] + (j // K) * W * H * 16 for j in range(n)]
            tracers[0].accumulate_images(pos, val, filter_params)
        return
    _run_threads(tracers, lambda i, t: t.render_images(first_seed, count, filter_params))
    for t in tracers:
        t.synchronize()


def prepare_pipelines(tracers, count: int) -> None:
    """prepare_images on every pipeline for a render_images_concurrently of `count` images: the
    whole count on banded pipelines, the largest per-pipeline share of a chunk on interleaved
    ones (each keeps only the images it renders)."""
    K = len(tracers)
    if K > 1 and getattr(tracers[0], "interleaved", False):
        chunk = min(count, K * max(1, min(getattr(t, "pool_images", 1) for t in tracers)))
        count = -(-chunk // K)
    for t in tracers:
        t.prepare_images(count)


def probe_row_cost(scene, first_seed: int = 1 << 20, images: int = 1, pool: int = 1 << 22, device: int = 0) -> np.ndarray:
    """Rays cast per film row over `images` images (seeds first_seed ..) of the whole film, from
    the tracer's row-cost probe: exact and schedule-independent, so every rank that probes the
    same scene gets the same vector and cuts the same balanced bands without communicating.
    (The default seeds lie outside any render's: the probe's image is not one of the film's.)"""
    t = WavefrontPathTracer(path_pool_size=pool, iterations_per_render=16, device=device)
    try:
        t.on_scene_loaded(scene)
        t.set_row_cost_probe(True)
        t.clear_film()
        t.render_images(first_seed, images)
        return t.read_row_cost().astype(np.int64)
    finally:
        t.destroy()
