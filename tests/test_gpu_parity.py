"""GPU parity: the gfx950 path (through the C ABI) against the CPU oracle.

Bar: integer state (RNG, hit indices, counters) is
bit-exact; the float outputs are also required bit-exact here because both
sides compile without contraction and with IEEE div/sqrt and share the same
deterministic transcendentals (DESIGN.md "Numerics"). Where a float
comparison is not bit-exact the tolerance is stated in the assertion.

The oracle side renders the scene flattened by the oracle ALONE (oracle.flat_with_own_bvh =
oracle.flatten_scene: its independent BVHAccel restatement over the scene's loaded meshes,
tests/test_bvh_pin.py, and its own lights, materials and instance arrays, tests/test_scene_pin.py)
with the oracle's own frame constants (oracle.frame_params), not with the product's flat scene.
"""
import numpy as np
import pytest

from conftest import MATERIAL_CASES, configure_lights, cornell

pytestmark = pytest.mark.gpu


def same_bits(a, b):
    """Bit-identical, except that a NaN matches any NaN: the reference's own arithmetic makes
    NaN (e.g. the power heuristic's inf/inf at grazing light samples), and the default NaN
    payload differs between x86 (sign set) and gfx950."""
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


def _rays(n, seed, room=True):
    from directcomputeraytracing_amd import make_rays
    rng = np.random.default_rng(seed)
    if room:
        o = rng.uniform([-1.4, 0.05, 1.05], [1.4, 1.95, 4.4], size=(n, 3))
    else:
        o = rng.uniform([-3, -1, -3], [3, 3, 0], size=(n, 3))
    d = rng.normal(size=(n, 3))
    d /= np.linalg.norm(d, axis=1, keepdims=True)
    # axis-aligned directions exercise the infinite-inverse slab path
    k = n // 16
    d[:k] = 0.0
    d[np.arange(k), rng.integers(0, 3, k)] = rng.choice([-1.0, 1.0], k)
    r = make_rays(o, d, 0.0, np.inf)
    r["t_max"][n // 2: n // 2 + n // 8] = rng.uniform(0.1, 2.0, n // 8)
    return r


def test_device_math_matches_oracle(gpu_tracer, oracle_mod):
    rng = np.random.default_rng(7)
    xs = [rng.uniform(-7, 7, 100000), rng.uniform(-100, 100, 20000), rng.uniform(-20, 20, 20000),
          rng.standard_normal(20000) * 1e-3, np.array([0.0, -0.0, 1.0, -1.0, 3.14159265, 1e-30, 88.0, -88.0])]
    x = np.concatenate(xs).astype(np.float32)
    for fn in range(5):
        y_gpu = gpu_tracer.math_eval(fn, x)
        y_cpu = oracle_mod.math_eval(fn, x)
        assert same_bits(y_gpu, y_cpu).all(), f"function {fn}"


def test_fast_reciprocal_equals_ieee_division(gpu_tracer):
    """rcp_ieee (dmath.h: v_rcp_f32 + one FMA Newton step on normal x with a normal reciprocal,
    the IEEE division otherwise) against IEEE 1/x -- numpy's float32 division on the host and the
    compiler's division on the GPU -- bit for bit: every exponent's edges and a stride through
    each binade, both signs, zeros, denormals, infinities and NaNs. (The exhaustive check of all
    4 227 858 432 fast-path inputs: tools/probe/rcp_exact.hip, profiles/r05_ab_rcp.txt.)"""
    rng = np.random.default_rng(11)
    e = np.arange(256, dtype=np.uint32)
    mant = np.concatenate([np.arange(0, 1 << 23, 4099, dtype=np.uint32),
                           np.array([0, 1, 2, (1 << 22), (1 << 23) - 2, (1 << 23) - 1], np.uint32)])
    bits = (e[:, None] << 23 | mant[None, :]).ravel()
    bits = np.concatenate([bits, bits | 0x80000000, rng.integers(0, 1 << 32, 1 << 21, dtype=np.uint64).astype(np.uint32)])
    x = bits.view(np.float32)
    with np.errstate(divide="ignore", over="ignore", invalid="ignore"):
        ref = (np.float32(1.0) / x).astype(np.float32)
    fast = gpu_tracer.math_eval(5, x)
    ieee = gpu_tracer.math_eval(6, x)
    assert same_bits(ieee, ref).all(), "the GPU's IEEE division differs from the host's"
    bad = ~same_bits(fast, ref)
    assert not bad.any(), f"{int(bad.sum())} of {x.size} differ, e.g. {bits[bad][:4]}"


def test_bxdf_luts_match_golden(gpu_tracer, golden_luts, oracle_mod):
    gpu = oracle_mod.luts_to_arrays(gpu_tracer.luts())
    ref = oracle_mod.luts_to_arrays(golden_luts)
    for k in ref:
        diff = np.abs(gpu[k].astype(np.int64) - ref[k].astype(np.int64))
        assert diff.max() == 0, f"{k}: {np.count_nonzero(diff)} texels differ, max {diff.max()} LSB"


@pytest.mark.parametrize("features", [0x0D, 0x05, 0x0F, 0x07])
def test_trace_rays_bit_exact(gpu_tracer, golden_luts, oracle_mod, features):
    s = cornell(64, 64, 2)
    gpu_tracer.on_scene_loaded(s)
    flat = oracle_mod.flat_with_own_bvh(s)
    for room in (True, False):
        rays = _rays(50000, 11 + features + room, room)
        h_gpu = gpu_tracer.trace_rays(rays, features)
        h_cpu, _ = oracle_mod.trace_rays(flat, rays, features)
        assert np.array_equal(h_gpu.view(np.uint8), h_cpu.view(np.uint8))
        o_gpu = gpu_tracer.occluded(rays, features)
        o_cpu, _ = oracle_mod.occluded(flat, rays, features)
        assert np.array_equal(o_gpu, o_cpu)


def _assert_cast_grid_resident(info):
    """The persistent cast grid holds no more workgroups per CU than the LDS does: gfx950
    allocates a workgroup's LDS in 1280-B granules (the HIP occupancy query rounds to 512 B, and
    a grid sized by it ran one workgroup per CU as a tail; tracer.hip LdsResident). Global-memory
    kernels: stack rows (traversal_stack + 2, or the spilling stack's LDS window) x block x 4 B +
    cached nodes x 32 + triangles x 48; the resident waves the info reports are that grid's."""
    if info["scene_in_lds"]:
        return
    cus = 256   # MI355X compute units (the cast grid is workgroups per CU x CUs)
    assert info["cast_grid"] % cus == 0, info["cast_grid"]
    per_cu = info["cast_grid"] // cus
    assert info["stack_lds_rows"] == (info["ring_rows"] or info["traversal_stack"] + 2)
    lds = info["stack_lds_rows"] * info["cast_block"] * 4 + info["cached_nodes"] * 32 + info["cached_triangles"] * 48
    assert per_cu >= 1 and per_cu * ((lds + 1279) // 1280 * 1280) <= 163840, (per_cu, lds)
    assert info["cast_waves_per_cu"] == per_cu * info["cast_block"] // 64


def _render_and_compare(tracer, oracle_mod, luts, scene, seeds):
    tracer.set_luts(luts)
    tracer.on_scene_loaded(scene)
    flat = oracle_mod.flat_with_own_bvh(scene)
    for seed in seeds:
        fr = scene.frame_params(seed)
        tracer.set_frame_params(fr)
        tracer.reset_image()
        for _ in range(10000):
            tracer.render()
            if tracer.is_image_complete():
                break
        assert tracer.is_image_complete()
        pos, val = tracer.read_samples()
        rng = tracer.read_rng()
        p_ref, v_ref, r_ref, c_ref = oracle_mod.render(flat, luts, oracle_mod.frame_params(scene, seed), oracle_mod.WAVEFRONT,
                                                        rng=True)
        assert np.array_equal(rng, r_ref), f"seed {seed}: RNG state differs at {np.count_nonzero((rng != r_ref).any(-1))} px"
        assert np.array_equal(pos.view(np.uint32), p_ref.view(np.uint32)), f"seed {seed}: sample positions"
        bad = np.count_nonzero(~same_bits(val, v_ref).all(-1))
        assert bad == 0, f"seed {seed}: {bad} pixels differ; max |d| {np.nanmax(np.abs(val - v_ref))}"
        c = tracer.counters()
        yield c, c_ref


def test_render_config1_bit_exact(gpu_tracer, golden_luts, oracle_mod):
    """configs[0]: Cornell box 128x128, 1 spp, maxBounce 2."""
    s = cornell(128, 128, 2)
    for c, c_ref in _render_and_compare(gpu_tracer, oracle_mod, golden_luts, s, [0]):
        pass


def test_render_8_bounces_odd_size_bit_exact(gpu_tracer, golden_luts, oracle_mod):
    """Ragged film (not a multiple of the 8x8 block), 8 bounces, several seeds."""
    s = cornell(133, 77, 8)
    list(_render_and_compare(gpu_tracer, oracle_mod, golden_luts, s, [0, 1, 5]))


@pytest.mark.parametrize("w,h,bounces", [(1, 1, 3), (1, 9, 2), (9, 1, 2), (17, 3, 0)])
def test_degenerate_films_bit_exact(native_lib, golden_luts, oracle_mod, w, h, bounces):
    """Edge sizes: a single pixel, one-column / one-row films (every 8x8 pixel block
    ragged), maxBounce 0 (CheckTermination after the camera ray only). Samples, RNG and
    the ray counts (WavefrontPathTracer.cpp:508-523 stats) equal the oracle's."""
    from directcomputeraytracing_amd import WavefrontPathTracer
    t = WavefrontPathTracer(path_pool_size=1 << 10, debug_rng=True)
    try:
        s = cornell(w, h, bounces)
        for c, c_ref in _render_and_compare(t, oracle_mod, golden_luts, s, [2]):
            assert c["extension_rays"] == c_ref["extension_rays"]
            assert c["shadow_rays"] == c_ref["shadow_rays"]
            assert c["new_paths"] == w * h
    finally:
        t.destroy()


def test_scene_without_lights_bit_exact(native_lib, golden_luts, oracle_mod):
    """lightCount 0: MATERIAL skips light sampling (no shadow rays), every sample is
    black, paths still bounce until termination (WavefrontPathTracing.hlsl:367-391)."""
    from directcomputeraytracing_amd import Scene, WavefrontPathTracer, scenes
    s = Scene((24, 16))
    s.reset(24, 16)
    s.load_from_file(scenes.CORNELL_OBJ)
    s.set_max_bounce(3)
    t = WavefrontPathTracer(path_pool_size=1 << 10, debug_rng=True)
    try:
        for c, c_ref in _render_and_compare(t, oracle_mod, golden_luts, s, [0]):
            assert c["shadow_rays"] == 0 and c_ref["shadow_rays"] == 0
            assert c["extension_rays"] == c_ref["extension_rays"]
        _, val = t.read_samples()
        assert not val[..., :3].any()
    finally:
        t.destroy()
    s.close()


def test_render_full_1080p_one_spp_bit_exact(native_lib, golden_luts, oracle_mod):
    """configs[1] resolution and depth: 1920x1080, 8 bounces, one image, whole film."""
    from directcomputeraytracing_amd import WavefrontPathTracer
    t = WavefrontPathTracer(path_pool_size=1 << 21, iterations_per_render=16, debug_rng=True)
    try:
        s = cornell(1920, 1080, 8)
        list(_render_and_compare(t, oracle_mod, golden_luts, s, [3]))
    finally:
        t.destroy()


def test_film_accumulation_matches_oracle(native_lib, golden_luts, oracle_mod):
    from directcomputeraytracing_amd import FILTER_BOX, FILTER_GAUSSIAN, FILTER_MITCHELL, FilterParams, \
        WavefrontPathTracer
    t = WavefrontPathTracer(path_pool_size=1 << 16)
    try:
        s = cornell(96, 64, 3)
        t.set_luts(golden_luts)
        t.on_scene_loaded(s)
        flat = oracle_mod.flat_with_own_bvh(s)
        for filt in (FilterParams(FILTER_BOX, 1.0, 1.5, 1 / 3, 1 / 3, 3),
                     FilterParams(FILTER_GAUSSIAN, 1.5, 2.0, 1 / 3, 1 / 3, 3),
                     FilterParams(FILTER_MITCHELL, 2.0, 1.5, 1 / 3, 1 / 3, 3)):
            t.clear_film()
            t.render_images(0, 3, filt)
            film = t.read_film()
            ref = np.zeros_like(film)
            for seed in range(3):
                p, v, _, _ = oracle_mod.render(flat, golden_luts, oracle_mod.frame_params(s, seed), oracle_mod.WAVEFRONT)
                oracle_mod.sample_convolution(filt, p, v, ref)
            assert same_bits(film, ref).all(), \
                f"filter {filt.filter}: max |d| {np.abs(film - ref).max()}"
    finally:
        t.destroy()


@pytest.mark.parametrize("case", range(12))
def test_film_random_filters_bit_exact(native_lib, golden_luts, oracle_mod, case):
    """SampleConvolution with seeded random filters on a ragged film (71 x 53, tiles cut by both
    edges): every kind (box, tent, gaussian, mitchell, lanczos) with random radii from 0.3 to 6 --
    the LDS-staged tiles and, past a 4-pixel halo, the direct gather -- and random gaussian
    alpha, Mitchell B / C and Lanczos tau; the film of two images equals the oracle's."""
    from directcomputeraytracing_amd import FilterParams, WavefrontPathTracer
    rng = np.random.default_rng(case)
    kind = case % 5
    radius = float(rng.uniform(0.3, 2.5) if case < 8 else rng.uniform(4.6, 6.0))
    filt = FilterParams(kind, radius, float(rng.uniform(0.5, 3.0)), float(rng.uniform(0, 1)), float(rng.uniform(0, 1)),
                        int(rng.integers(1, 5)))
    s = cornell(71, 53, 2)
    t = WavefrontPathTracer(path_pool_size=1 << 14)
    try:
        t.set_luts(golden_luts)
        t.on_scene_loaded(s)
        t.clear_film()
        t.render_images(3, 2, filt)
        film = t.read_film()
    finally:
        t.destroy()
    flat = oracle_mod.flat_with_own_bvh(s)
    ref = np.zeros_like(film)
    for seed in (3, 4):
        p, v, _, _ = oracle_mod.render(flat, golden_luts, oracle_mod.frame_params(s, seed), oracle_mod.WAVEFRONT)
        oracle_mod.sample_convolution(filt, p, v, ref)
    bad = np.count_nonzero(~same_bits(film, ref).all(-1))
    assert bad == 0, f"filter {kind} r {radius}: {bad} pixels differ"


def test_film_radius_just_below_half_integer(native_lib, golden_luts, oracle_mod):
    """A pixel's window [floor(c - r), floor(c + r)] reaches floor(r + 0.5) + 1 pixels out where
    c + r rounds up to an integer (r = nextafter(1.5, 0) at c = 100.5): the LDS-staged film pass
    stages each tile's exact window union, so such films stay bit-exact (odd film size: partial tiles)."""
    from directcomputeraytracing_amd import FILTER_BOX, FILTER_GAUSSIAN, FILTER_TRIANGLE, FilterParams, \
        WavefrontPathTracer
    below = lambda x: float(np.nextafter(np.float32(x), np.float32(0)))
    t = WavefrontPathTracer(path_pool_size=1 << 15)
    try:
        s = cornell(150, 70, 2)
        t.set_luts(golden_luts)
        t.on_scene_loaded(s)
        flat = oracle_mod.flat_with_own_bvh(s)
        for filt in (FilterParams(FILTER_BOX, below(1.5), 1.5, 1 / 3, 1 / 3, 3),
                     FilterParams(FILTER_TRIANGLE, below(1.5), 1.5, 1 / 3, 1 / 3, 3),
                     FilterParams(FILTER_GAUSSIAN, below(2.5), 2.0, 1 / 3, 1 / 3, 3),
                     FilterParams(FILTER_BOX, below(4.5), 1.5, 1 / 3, 1 / 3, 3)):
            t.clear_film()
            t.render_images(0, 2, filt)
            film = t.read_film()
            ref = np.zeros_like(film)
            for seed in range(2):
                p, v, _, _ = oracle_mod.render(flat, golden_luts, oracle_mod.frame_params(s, seed), oracle_mod.WAVEFRONT)
                oracle_mod.sample_convolution(filt, p, v, ref)
            assert same_bits(film, ref).all(), f"filter {filt.filter} r={filt.radius!r}"
    finally:
        t.destroy()


def test_film_partition_halo_for_radius_just_below_half_integer(native_lib, golden_luts):
    """Partitioned films with r = nextafter(1.5, 0): the window reaches 2 rows out, so the partition
    needs halo_for_radius(r) = 2 rows (1 is refused), and the rank films then sum to the 1-GPU film."""
    from directcomputeraytracing_amd import DCRTError, FILTER_BOX, FilterParams, WavefrontPathTracer
    from directcomputeraytracing_amd.partition import halo_for_radius
    r = float(np.nextafter(np.float32(1.5), np.float32(0)))
    filt = FilterParams(FILTER_BOX, r, 1.5, 1 / 3, 1 / 3, 3)
    s = cornell(96, 120, 2)
    halo = halo_for_radius(r, 120)
    assert halo == 2
    films = []
    for world, rank, h in [(1, 0, 0), (3, 0, halo), (3, 1, halo), (3, 2, halo), (3, 1, 1)]:
        t = WavefrontPathTracer(path_pool_size=1 << 15)
        try:
            t.set_luts(golden_luts)
            t.on_scene_loaded(s)
            t.set_film_partition(world, rank, 16, h)
            t.clear_film()
            if h == 1:
                with pytest.raises(DCRTError):
                    t.render_images(0, 2, filt)
                continue
            t.render_images(0, 2, filt)
            films.append(t.read_film())
        finally:
            t.destroy()
    assert same_bits(films[1] + films[2] + films[3], films[0]).all()


def test_material_variant_matches_generic(native_lib, golden_luts, monkeypatch):
    """The Cornell scene (diffuse/plastic, point light) runs the capability-specialised MATERIAL
    variant (material_kernel<kCapOpaqueDelta>); forcing the generic variant gives the same bits
    (samples, RNG states and film)."""
    from directcomputeraytracing_amd import WavefrontPathTracer
    s = cornell(128, 72, 6)
    out = []
    for generic in ("0", "1"):
        monkeypatch.setenv("DCRT_MATERIAL_GENERIC", generic)
        t = WavefrontPathTracer(path_pool_size=1 << 14, debug_rng=True)
        try:
            t.set_luts(golden_luts)
            t.on_scene_loaded(s)
            t.clear_film()
            t.render_images(3, 2)
            out.append((t.read_samples(), t.read_rng(), t.read_film()))
        finally:
            t.destroy()
    (p0, v0), r0, f0 = out[0]
    (p1, v1), r1, f1 = out[1]
    assert np.array_equal(r0, r1)
    assert same_bits(p0, p1).all() and same_bits(v0, v1).all() and same_bits(f0, f1).all()


def test_film_partition_sums_to_single_gpu(native_lib, golden_luts):
    """Stripes + halo per rank: the rank films sum to the 1-GPU film exactly."""
    from directcomputeraytracing_amd import WavefrontPathTracer
    s = cornell(160, 120, 3)
    films = []
    for world, rank in [(1, 0), (3, 0), (3, 1), (3, 2)]:
        t = WavefrontPathTracer(path_pool_size=1 << 15)
        try:
            t.set_luts(golden_luts)
            t.on_scene_loaded(s)
            t.set_film_partition(world, rank, 16)
            t.clear_film()
            t.render_images(0, 2)
            films.append(t.read_film())
        finally:
            t.destroy()
    total = films[1] + films[2] + films[3]
    assert same_bits(total, films[0]).all()


def test_row_cost_probe_matches_oracle(native_lib, golden_luts, oracle_mod):
    """The row-cost probe (MATERIAL's PROBE variant): rays cast per film row over two images --
    every extension ray the wavefront shades plus every shadow ray it casts -- equal the oracle's
    per-row counts exactly; on a tracer with film bands, the rows it path-traces (bands + halo)
    carry their counts and the other rows none. Turning it off restores the shipped kernels."""
    from directcomputeraytracing_amd import WavefrontPathTracer
    W, H = 160, 96
    s = cornell(W, H, 4)
    flat = oracle_mod.flat_with_own_bvh(s)
    ref = np.zeros(H, np.int64)
    for seed in (3, 4):
        fr = oracle_mod.frame_params(s, seed)
        for y in range(H):
            _, _, _, c = oracle_mod.render(flat, golden_luts, fr, oracle_mod.WAVEFRONT, rect=(0, y, W, 1))
            ref[y] += c["extension_rays"] + c["shadow_rays"]
    t = WavefrontPathTracer(path_pool_size=1 << 14)
    try:
        t.set_luts(golden_luts)
        t.on_scene_loaded(s)
        t.set_row_cost_probe(True)
        t.clear_film()
        t.render_images(3, 2)
        rows = t.read_row_cost()
        c = t.counters()
        assert np.array_equal(rows.astype(np.int64), ref)
        assert rows.sum() == c["extension_rays"] + c["shadow_rays"]
        t.set_film_bands([(10, 37), (60, 61)], 2)     # the counters restart with the new rows
        t.clear_film()
        t.render_images(3, 2)
        banded = t.read_row_cost().astype(np.int64)
        traced = np.zeros(H, bool)
        traced[8:39] = traced[58:63] = True
        assert np.array_equal(banded[traced], ref[traced]) and not banded[~traced].any()
        t.set_row_cost_probe(False)
        t.set_film_partition(1, 0, 64)
        t.clear_film()
        t.render_images(3, 2)
        with pytest.raises(Exception, match="probe is off"):
            t.read_row_cost()
    finally:
        t.destroy()


def test_balanced_bands_pipelines_sum_to_oracle_film(native_lib, golden_luts, oracle_mod):
    """bench.py's default construction with cost-balanced bands (make_pipelines(row_cost=
    probe_row_cost(scene))): three pipelines on one GPU, and a world of four ranks with two
    pipelines each -- every rank's pipeline films summed, then the ranks summed -- give the
    oracle's film bit for bit. The bands are uneven (equal cost, not equal height)."""
    from directcomputeraytracing_amd import make_pipelines, probe_row_cost
    from directcomputeraytracing_amd.partition import balanced_bands, halo_for_radius
    W, H = 160, 96
    s = cornell(W, H, 4)
    filt = s.filter_params()
    cost = probe_row_cost(s)
    assert cost.sum() > W * H
    heights = {b[1] - b[0] for b in balanced_bands(cost, 8, max(1, halo_for_radius(filt.radius, H)))}
    assert len(heights) > 1
    flat = oracle_mod.flat_with_own_bvh(s)
    ref = np.zeros((H, W, 4), np.float32)
    for seed in range(2):
        p, v, _, _ = oracle_mod.render(flat, golden_luts, oracle_mod.frame_params(s, seed), oracle_mod.WAVEFRONT)
        oracle_mod.sample_convolution(filt, p, v, ref)
    for world, K in ((1, 3), (4, 2)):
        total = np.zeros_like(ref)
        for rank in range(world):
            ts = make_pipelines(s, 1 << 15, streams=K, images=2, world=world, rank=rank, row_cost=cost)
            try:
                for t in ts:
                    t.set_luts(golden_luts)
                    t.clear_film()
                render_images_concurrently_local(ts, 0, 2, filt)
                for t in ts:
                    total += t.read_film()
            finally:
                for t in ts:
                    t.destroy()
        assert same_bits(total, ref).all(), (world, K)


@pytest.mark.parametrize("pool", [1 << 16, 1 << 14])
def test_interleaved_pipelines_match_oracle_film(native_lib, golden_luts, oracle_mod, pool):
    """Pipelines that split the IMAGES of a GPU's rows instead of the rows (make_pipelines(
    interleave=True)): pipeline s renders images s, s + K, ... (seed stride K) without the film
    pass, and pipeline 0 convolves every image in image order from the K pipelines' sample
    textures (accumulate_images). One GPU with three pipelines, and four ranks of two pipelines
    on one or two cost-balanced bands each: the film (summed over the ranks) is the oracle's bit
    for bit, and the other pipelines' films stay empty. The small pool forces chunks of one
    image per pipeline (several batches, each with its virtual start)."""
    from directcomputeraytracing_amd import make_pipelines, probe_row_cost, render_images_concurrently
    W, H, images = 160, 96, 5
    s = cornell(W, H, 4)
    filt = s.filter_params()
    cost = probe_row_cost(s)
    flat = oracle_mod.flat_with_own_bvh(s)
    ref = np.zeros((H, W, 4), np.float32)
    for seed in range(images):
        p, v, _, _ = oracle_mod.render(flat, golden_luts, oracle_mod.frame_params(s, seed), oracle_mod.WAVEFRONT)
        oracle_mod.sample_convolution(filt, p, v, ref)
    for world, K, B in ((1, 3, 0), (4, 2, 1), (4, 2, 2)):
        total = np.zeros_like(ref)
        for rank in range(world):
            ts = make_pipelines(s, pool * K, streams=K, images=images, world=world, rank=rank, row_cost=cost,
                                interleave=True, bands_per_rank=B)
            try:
                for t in ts:
                    t.set_luts(golden_luts)
                    t.clear_film()
                render_images_concurrently(ts, 0, images, filt)
                total += ts[0].read_film()
                for t in ts[1:]:
                    assert not t.read_film().any()
                assert sum(t.counters()["images_completed"] for t in ts) == images
            finally:
                for t in ts:
                    t.destroy()
        assert same_bits(total, ref).all(), (world, K, B)


def render_images_concurrently_local(ts, first, count, filt):
    from directcomputeraytracing_amd import render_images_concurrently
    render_images_concurrently(ts, first, count, filt)


def test_image_batches_match_single_images(native_lib, golden_luts, oracle_mod):
    """render_images in batches (images sharing the path pool) == one image at a time:
    same film bits, and read_samples returns the last image's samples."""
    from directcomputeraytracing_amd import WavefrontPathTracer
    s = cornell(96, 64, 4)
    films, samples = [], []
    for batch in (1, 2, 0):
        t = WavefrontPathTracer(path_pool_size=1 << 12, debug_rng=True)
        try:
            t.set_luts(golden_luts)
            t.on_scene_loaded(s)
            t.set_image_batch(batch)
            if batch == 2:
                t.prepare_images(3)    # allocate + capture ahead: same bits
            t.clear_film()
            t.render_images(5, 3)
            films.append(t.read_film())
            samples.append(t.read_samples())
            c = t.counters()
            assert c["images_completed"] == 3 and c["new_paths"] == 3 * 96 * 64
        finally:
            t.destroy()
    for f in films[1:]:
        assert same_bits(f, films[0]).all()
    p_ref, v_ref, _, _ = oracle_mod.render(oracle_mod.flat_with_own_bvh(s), golden_luts, oracle_mod.frame_params(s, 7), oracle_mod.WAVEFRONT)
    for pos, val in samples:
        assert same_bits(pos, p_ref).all() and same_bits(val, v_ref).all()


@pytest.mark.parametrize("cached", [True, False])
def test_identity_cast_kernel_bit_exact(native_lib, golden_luts, monkeypatch, cached):
    """The cast kernel without instance space (every instance's inverse exactly the identity, as
    for every OBJ shape: IDENT in dscene.h) against the kernel that keeps it (DCRT_IDENT_CAST=0),
    as the cache-only kernel and (DCRT_NO_LDS_CACHE=1) as the global-memory one -- and the cache-only
    one over the entry-free node order (FLAT, tracer.hip EntryFreeLayout: cast_identity 2) against
    it over PackBVH's (DCRT_FLAT_CAST=0): the same samples, RNG state, film and ray counts bit for
    bit, and the instrumented traversal counts (node visits, triangle tests, BLAS entries) equal."""
    from directcomputeraytracing_amd import FILTER_BOX, FilterParams, WavefrontPathTracer
    monkeypatch.setenv("DCRT_NO_LDS_CACHE", "0" if cached else "1")
    s = cornell(96, 64, 6)
    filt = FilterParams(FILTER_BOX, 1.0, 1.5, 1 / 3, 1 / 3, 3)
    runs = {}
    for ident in ("1", "0", "1-noflat"):
        monkeypatch.setenv("DCRT_IDENT_CAST", ident[0])
        monkeypatch.setenv("DCRT_FLAT_CAST", "0" if ident.endswith("noflat") else "1")
        t = WavefrontPathTracer(path_pool_size=1 << 14, debug_rng=True)
        try:
            t.set_luts(golden_luts)
            t.on_scene_loaded(s)
            info = t.info()
            want = 0 if ident == "0" else (2 if cached and ident == "1" else 1)
            assert info["scene_in_lds"] == (1 if cached else 0) and info["cast_identity"] == want, info
            _assert_cast_grid_resident(info)
            t.clear_film()
            t.render_images(0, 3, filt)
            film, samples, rng, c = t.read_film(), t.read_samples(), t.read_rng(), t.counters()
            t.set_instrumentation(True, False)
            t.reset_stats()
            t.render_images(0, 2, filt)
            st = t.traversal_stats()
            runs[ident] = (film, samples, rng, c, {k: st[k] for k in st if k.endswith(("visits", "tests", "entries"))})
        finally:
            t.destroy()
    for other in ("0", "1-noflat"):
        (fa, (pa, va), ra, ca, sa), (fb, (pb, vb), rb, cb, sb) = runs["1"], runs[other]
        assert np.array_equal(ra, rb) and same_bits(pa, pb).all() and same_bits(va, vb).all() and same_bits(fa, fb).all()
        assert ca["extension_rays"] == cb["extension_rays"] and ca["shadow_rays"] == cb["shadow_rays"]
        assert sa == sb and sa["ext_node_visits"] > 0


@pytest.mark.parametrize("scene_name", ["cornell", "xml_mix"])
def test_material_lds_scene_copy_bit_exact(native_lib, golden_luts, monkeypatch, scene_name):
    """MATERIAL's LDS scene copy (material_kernel<CAPS, 1>: triangles, forward transforms,
    instance words, materials and lights read from LDS; <CAPS, 2>: all but the triangles)
    against the global-memory variant (DCRT_MATERIAL_LDS=0): the same samples, RNG state and
    film bit for bit; the whole copy is what the default picks for these small scenes, the
    partial one what it picks for the larger config scenes (the other parity tests compare
    both with the oracle)."""
    from conftest import GOLDEN
    from directcomputeraytracing_amd import FILTER_BOX, FilterParams, Scene, WavefrontPathTracer
    if scene_name == "cornell":
        s = cornell(96, 64, 6)
    else:
        s = Scene((45, 29))
        s.load_from_file(GOLDEN / "xml_mix" / "scene.xml")
    filt = FilterParams(FILTER_BOX, 1.0, 1.5, 1 / 3, 1 / 3, 3)
    runs, sizes = {}, {}
    # 16 KiB: the whole copy; 1 KiB: all but the triangles (the partial copy larger scenes get);
    # 0: none
    for budget in ("16384", "1024", "0"):
        monkeypatch.setenv("DCRT_MATERIAL_LDS", budget)
        t = WavefrontPathTracer(path_pool_size=1 << 14, debug_rng=True)
        try:
            t.set_luts(golden_luts)
            t.on_scene_loaded(s)
            sizes[budget] = t.info()["material_lds"]
            t.clear_film()
            t.render_images(0, 3, filt)
            runs[budget] = (t.read_film(), t.read_samples(), t.read_rng())
        finally:
            t.destroy()
    assert sizes["16384"] > sizes["1024"] > 0 and sizes["0"] == 0
    fb, (pb, vb), rb = runs["0"]
    for budget in ("16384", "1024"):
        fa, (pa, va), ra = runs[budget]
        assert np.array_equal(ra, rb) and same_bits(pa, pb).all() and same_bits(va, vb).all() and same_bits(fa, fb).all(), budget


@pytest.mark.parametrize("cache,scene_name,pool", [("lds", "cornell", 1 << 15), ("global", "cornell", 1 << 15),
                                                   ("pair", "cornell", 1 << 12), ("global", "xml_mix", 1 << 14),
                                                   ("pair", "xml_mix", 3000)])
def test_virtual_batch_start_bit_exact(native_lib, golden_luts, oracle_mod, monkeypatch, cache, scene_name, pool):
    """Virtual batch starts (control_kernel: the cast generates the camera rays of a batch's
    statically claimed slots, the first MATERIAL pass recomputes NEW_PATH's rng) on the
    global-memory and pair cast kernels, with drain completion (drain_kernel): a ragged film
    (holes in the virtual queue), several batches, pools smaller than a batch (the rest of the
    blocks claimed later), against the oracle (samples, RNG state, film, ray counts) and
    against DCRT_VIRTUAL_START=0 DCRT_DRAIN_PATHS=0."""
    from conftest import GOLDEN
    from directcomputeraytracing_amd import FILTER_BOX, FilterParams, Scene, WavefrontPathTracer
    monkeypatch.setenv("DCRT_NO_LDS_CACHE", "0" if cache == "lds" else "1")
    monkeypatch.setenv("DCRT_PAIR_TRAVERSAL", "1" if cache == "pair" else "0")
    if scene_name == "cornell":
        s = cornell(133, 77, 6)
    else:
        s = Scene((45, 29))
        s.load_from_file(GOLDEN / "xml_mix" / "scene.xml")
    W, H = s.resolution
    filt = FilterParams(FILTER_BOX, 1.0, 1.5, 1 / 3, 1 / 3, 3)
    runs = {}
    # virtual start + drain completion (every path of a batch completed in drain_kernel once at
    # most 400 remain) against neither
    for virtual, drain in (("1", "400"), ("0", "0")):
        monkeypatch.setenv("DCRT_VIRTUAL_START", virtual)
        monkeypatch.setenv("DCRT_DRAIN_PATHS", drain)
        t = WavefrontPathTracer(path_pool_size=pool, debug_rng=True)
        try:
            t.set_luts(golden_luts)
            t.on_scene_loaded(s)
            t.set_image_batch(2)
            t.clear_film()
            t.render_images(3, 5, filt)
            runs[virtual] = (t.read_film(), t.read_samples(), t.read_rng(), t.counters())
        finally:
            t.destroy()
    film, (pos, val), rng, c = runs["1"]
    flat = oracle_mod.flat_with_own_bvh(s)
    ref = np.zeros_like(film)
    ext = shadow = 0
    for seed in range(3, 8):
        p, v, r, cr = oracle_mod.render(flat, golden_luts, oracle_mod.frame_params(s, seed), oracle_mod.WAVEFRONT, rng=True)
        oracle_mod.sample_convolution(filt, p, v, ref)
        ext += cr["extension_rays"]
        shadow += cr["shadow_rays"]
    assert np.array_equal(rng, r) and same_bits(pos, p).all() and same_bits(val, v).all()   # the last image
    assert same_bits(film, ref).all()
    assert c["extension_rays"] == ext and c["shadow_rays"] == shadow and c["new_paths"] == 5 * W * H
    assert same_bits(runs["0"][0], film).all() and runs["0"][3]["extension_rays"] == ext


def test_concurrent_stream_partitions_sum_to_single_film(native_lib, golden_luts):
    """bench --streams 2: two tracers on one GPU render their bands concurrently (two host
    threads, two streams); add_film_device of one film into the other == 1-tracer film."""
    from directcomputeraytracing_amd import WavefrontPathTracer, render_images_concurrently
    from directcomputeraytracing_amd.partition import stream_partition
    s = cornell(160, 120, 3)
    ref = WavefrontPathTracer(path_pool_size=1 << 15)
    try:
        ref.set_luts(golden_luts)
        ref.on_scene_loaded(s)
        ref.clear_film()
        ref.render_images(0, 3)
        want = ref.read_film()
    finally:
        ref.destroy()
    ts = []
    try:
        for k in range(2):
            t = WavefrontPathTracer(path_pool_size=1 << 14)
            t.set_luts(golden_luts)
            t.on_scene_loaded(s)
            w, v, sh = stream_partition(120, 1, 0, 2, k, 64)
            t.set_film_partition(w, v, sh)
            t.clear_film()
            ts.append(t)
        render_images_concurrently(ts, 0, 3)
        ts[0].add_film_device(ts[1].film_device_ptr())
        assert same_bits(ts[0].read_film(), want).all()
    finally:
        for t in ts:
            t.destroy()


def test_tiny_pool_renders_every_pixel(native_lib, golden_luts, oracle_mod):
    """A pool smaller than one CONTROL workgroup per pixel-block shard is grown to it:
    every shard's pixel blocks get claimed and the image completes bit-exact."""
    from directcomputeraytracing_amd import WavefrontPathTracer
    s = cornell(40, 24, 2)
    t = WavefrontPathTracer(path_pool_size=300)
    try:
        t.set_luts(golden_luts)
        t.on_scene_loaded(s, frame_seed=4)
        t.clear_film()
        t.render_images(4, 1)
        pos, val = t.read_samples()
    finally:
        t.destroy()
    p_ref, v_ref, _, _ = oracle_mod.render(oracle_mod.flat_with_own_bvh(s), golden_luts, oracle_mod.frame_params(s, 4), oracle_mod.WAVEFRONT)
    assert same_bits(pos, p_ref).all() and same_bits(val, v_ref).all()


def test_partition_rejects_filter_wider_than_halo(native_lib, golden_luts):
    from directcomputeraytracing_amd import DCRTError, FILTER_BOX, FilterParams, WavefrontPathTracer
    s = cornell(64, 48, 2)
    t = WavefrontPathTracer(path_pool_size=1 << 12)
    try:
        t.set_luts(golden_luts)
        t.on_scene_loaded(s)
        t.set_film_partition(2, 0, 16, 1)
        with pytest.raises(DCRTError):
            t.render_images(0, 1, FilterParams(FILTER_BOX, 2.0, 1.5, 1 / 3, 1 / 3, 3))
        t.render_images(0, 1, FilterParams(FILTER_BOX, 1.0, 1.5, 1 / 3, 1 / 3, 3))
    finally:
        t.destroy()


@pytest.mark.parametrize("scene_name,order", [("cornell", "flat"), ("cornell", "pairs"), ("xml_mix", "pairs")])
def test_traversal_counters_match_oracle(native_lib, golden_luts, oracle_mod, monkeypatch, scene_name, order):
    """Instrumented casts count the same AABB/triangle/BLAS work as the oracle (bytes/ray basis),
    on PackBVH's node order and on the device's child-pair order (the pair traversal's scenes:
    forced here with the LDS cache off; the counting kernel reads the order from the scene)."""
    from conftest import GOLDEN
    from directcomputeraytracing_amd import Scene, WavefrontPathTracer
    if order == "pairs":
        monkeypatch.setenv("DCRT_NO_LDS_CACHE", "1")
        monkeypatch.setenv("DCRT_PAIR_TRAVERSAL", "1")
    t = WavefrontPathTracer(path_pool_size=1 << 16)
    try:
        if scene_name == "cornell":
            s = cornell(128, 96, 4)
        else:
            s = Scene((64, 48))
            s.load_from_file(GOLDEN / "xml_mix" / "scene.xml")
        t.set_luts(golden_luts)
        t.on_scene_loaded(s)
        assert t.info()["pair_traversal"] == (1 if order == "pairs" else 0)
        t.set_instrumentation(True, True)
        t.reset_stats()
        t.render_images(2, 1)
        st = t.traversal_stats()
        c = t.counters()
        _, _, _, ref = oracle_mod.render(oracle_mod.flat_with_own_bvh(s), golden_luts, oracle_mod.frame_params(s, 2), oracle_mod.WAVEFRONT)
        assert c["extension_rays"] == ref["extension_rays"]
        assert c["shadow_rays"] == ref["shadow_rays"]
        assert st["ext_node_visits"] == ref["node_visits"]
        assert st["ext_triangle_tests"] == ref["triangle_tests"]
        assert st["ext_blas_entries"] == ref["blas_entries"]
        assert st["shadow_node_visits"] == ref["shadow_node_visits"]
        assert st["shadow_triangle_tests"] == ref["shadow_triangle_tests"]
        assert st["shadow_blas_entries"] == ref["shadow_blas_entries"]
        assert st["ext_launches"] > 0 and st["ext_kernel_ms"] > 0
    finally:
        t.destroy()


def test_missing_scene_fails_loudly(native_lib):
    from directcomputeraytracing_amd import DCRTError, WavefrontPathTracer
    t = WavefrontPathTracer(path_pool_size=1 << 12)
    try:
        with pytest.raises(DCRTError):
            t.render()
    finally:
        t.destroy()


# ---- BSDF / light coverage: every material type and light type, GPU vs oracle ----------
@pytest.mark.parametrize("case", sorted(MATERIAL_CASES))
def test_materials_bit_exact(gpu_tracer, golden_luts, oracle_mod, case):
    s = cornell(48, 40, 5)
    for args in MATERIAL_CASES[case]:
        s.set_material(*args)
    list(_render_and_compare(gpu_tracer, oracle_mod, golden_luts, s, [0, 3]))


@pytest.mark.parametrize("env", ["constant", "cube", "directional"])
def test_lights_bit_exact(gpu_tracer, golden_luts, oracle_mod, env):
    s = cornell(48, 40, 4)
    configure_lights(s, env)     # the room is open towards the camera: escaping rays see the sky
    list(_render_and_compare(gpu_tracer, oracle_mod, golden_luts, s, [1, 2]))


def test_pinhole_and_filters(gpu_tracer, golden_luts, oracle_mod):
    s = cornell(40, 40, 3)
    s.set_lens(camera_type=0, fov_x=1.0)
    list(_render_and_compare(gpu_tracer, oracle_mod, golden_luts, s, [4]))


def test_xml_scene_mesh_lights_bit_exact(gpu_tracer, golden_luts, oracle_mod):
    """Mitsuba XML fixture: area (triangle) light, env + directional, twosided roughplastic,
    roughconductor, roughdielectric, instanced OBJ, shared rectangle, thin lens."""
    from conftest import GOLDEN
    from directcomputeraytracing_amd import Scene
    s = Scene((32, 32))
    s.load_from_file(GOLDEN / "xml_mix" / "scene.xml")
    list(_render_and_compare(gpu_tracer, oracle_mod, golden_luts, s, [0, 7]))


@pytest.mark.parametrize("cache", ["lds", "lds-nomerge", "global", "pair"])
@pytest.mark.parametrize("features", [0x05, 0x0F, 0x07])
@pytest.mark.parametrize("scene_name", ["cornell", "xml_mix"])
def test_traversal_variants_wavefront_bit_exact(native_lib, golden_luts, oracle_mod, monkeypatch, scene_name, features, cache):
    """The merged cast kernel's traversal variants through the whole wavefront path:
    Moller-Trumbore (WATERTIGHT off), BVH_NO_FRONT_TO_BACK_TRAVERSAL, both; the cache-only
    kernel (scene, permuted triangle copies and instance transforms in LDS: both scenes
    fit; Cornell's over the entry-free node order, its TLAS leaves merged with their BLAS roots
    or -- lds-nomerge -- every one over an empty node), the global-memory kernel
    (DCRT_NO_LDS_CACHE) and the global-memory kernel with the pair-expanding traversal
    (trav_visit_pair). xml_mix has transformed rectangle instances (instance-space rays in the
    BLAS)."""
    from conftest import GOLDEN
    from directcomputeraytracing_amd import Scene, WavefrontPathTracer
    if cache == "lds-nomerge":
        monkeypatch.setenv("DCRT_FLAT_MERGE", "0")
    if cache in ("global", "pair"):
        monkeypatch.setenv("DCRT_NO_LDS_CACHE", "1")
    monkeypatch.setenv("DCRT_PAIR_TRAVERSAL", "1" if cache == "pair" else "0")
    if scene_name == "cornell":
        s = cornell(64, 48, 6)
    else:
        s = Scene((32, 32))
        s.load_from_file(GOLDEN / "xml_mix" / "scene.xml")
    s.features = features
    t = WavefrontPathTracer(path_pool_size=1 << 12, debug_rng=True)
    try:
        list(_render_and_compare(t, oracle_mod, golden_luts, s, [0, 3]))
        assert t.info()["pair_traversal"] == (1 if cache == "pair" else 0)
        if scene_name == "cornell" and cache.startswith("lds"):
            assert t.info()["cast_identity"] == 2   # (the entry-free order)
    finally:
        t.destroy()


@pytest.mark.parametrize("name,cube,ms", [("coffee", True, True), ("coffee", True, False), ("spaceship", False, False),
                                          ("lamp", False, False)])
def test_config_scenes_bit_exact(gpu_tracer, golden_luts, oracle_mod, name, cube, ms):
    """configs[2..4] (coffee / spaceship / lamp, procedural XML fixtures) at 160x90, 8 bounces;
    coffee as configs[2] names it (Kulla-Conty multiscattering on every plastic, conductor and
    dielectric material) and as the loader leaves it (off)."""
    from test_oracle import load_fixture_scene
    s = load_fixture_scene(name, env_cube=cube, multiscattering=ms)
    list(_render_and_compare(gpu_tracer, oracle_mod, golden_luts, s, [0, 1]))
    _assert_cast_grid_resident(gpu_tracer.info())


@pytest.mark.parametrize("framing,ring", [("wide", None), ("close", None), ("close", "8")])
def test_full_size_spaceship_mesh_bit_exact(gpu_tracer, golden_luts, oracle_mod, tmp_path, monkeypatch, framing, ring):
    """configs[3] at its full mesh size (261 120 triangles x 8 instances, 522 k BVH nodes,
    stack depth 30: most nodes outside the LDS scene cache), 320x180, 8 bounces, 1 spp; both
    framings (the close one: hulls fill the frame, paths bounce between them). The scene's
    default is the spilling stack (a 16-row LDS window over per-lane global columns: 6 instead
    of 4 workgroups per CU); ring "8" forces an 8-row window, so most deep entries spill and
    come back (ring_maintain): ring_spills() > 0."""
    from directcomputeraytracing_amd import Scene, scenes
    if ring:
        monkeypatch.setenv("DCRT_STACK_RING", ring)
    s = Scene((320, 180))
    s.load_from_file(scenes.write_spaceship(tmp_path, 320, 180, nu=512, nv=256, ships=8, framing=framing))
    assert s.bvh_info()["total_nodes"] > 500_000
    list(_render_and_compare(gpu_tracer, oracle_mod, golden_luts, s, [3]))
    info = gpu_tracer.info()
    assert info["pair_traversal"] == 1   # (beyond an XCD's L2: trav_visit_pair)
    assert info["ring_rows"] == int(ring or 16) and info["stack_lds_rows"] == info["ring_rows"]
    assert info["cast_waves_per_cu"] >= 24 if ring is None else True
    if ring == "8":
        # (the 16-row default spills only the rare lanes more than 13 entries deep, which this
        # small image may or may not have; an 8-row window spills on every deep descent)
        assert gpu_tracer.ring_spills() > 0
    _assert_cast_grid_resident(info)


@pytest.mark.parametrize("kernel", ["pair", "global", "ident", "split"])
@pytest.mark.parametrize("scene_name", ["cornell", "xml_mix"])
def test_stack_ring_and_split_casts_bit_exact(native_lib, golden_luts, oracle_mod, monkeypatch, scene_name, kernel):
    """The spilling traversal stack forced onto small scenes (DCRT_STACK_RING=8: an 8-row LDS
    window, entries beyond it in per-lane global columns) in the pair, global-memory and
    identity-space (IDENT) cast kernels, and the reference's two separate cast kernels
    (DCRT_SPLIT_CASTS=1: extension_kernel, then shadow_kernel, whole stack): samples, RNG
    state and ray counts against the oracle."""
    from conftest import GOLDEN
    from directcomputeraytracing_amd import Scene, WavefrontPathTracer
    monkeypatch.setenv("DCRT_NO_LDS_CACHE", "1")
    monkeypatch.setenv("DCRT_PAIR_TRAVERSAL", "1" if kernel == "pair" else "0")
    monkeypatch.setenv("DCRT_IDENT_CAST", "1" if kernel == "ident" else "0")
    if kernel == "split":
        monkeypatch.setenv("DCRT_SPLIT_CASTS", "1")
    else:
        monkeypatch.setenv("DCRT_STACK_RING", "8")
    if scene_name == "cornell":
        s = cornell(96, 64, 8)
    else:
        s = Scene((48, 40))
        s.load_from_file(GOLDEN / "xml_mix" / "scene.xml")
    t = WavefrontPathTracer(path_pool_size=1 << 13, debug_rng=True)
    try:
        rays = [0, 0]
        for c, c_ref in _render_and_compare(t, oracle_mod, golden_luts, s, [0, 5]):
            rays = [rays[0] + c_ref["extension_rays"], rays[1] + c_ref["shadow_rays"]]   # (the tracer's counts accumulate)
            assert [c["extension_rays"], c["shadow_rays"]] == rays
        info = t.info()
        assert info["pair_traversal"] == (1 if kernel == "pair" else 0)
        assert info["ring_rows"] == (0 if kernel == "split" else 8)
        if kernel == "ident":
            assert info["cast_identity"] == (1 if scene_name == "cornell" else 0)   # (the ring kernel: not cache-only)
    finally:
        t.destroy()


@pytest.mark.parametrize("scene_name", ["cornell", "xml_mix"])
def test_pair_order_trace_rays_and_megakernel_bit_exact(native_lib, golden_luts, oracle_mod, monkeypatch, scene_name):
    """The kernels that read the node order from the scene (trace_rays' batch kernel, the
    megakernel) on the child-pair order (tracer.hip PairLayout: forced here with the LDS cache
    off), against the oracle on PackBVH's order."""
    from conftest import GOLDEN
    from directcomputeraytracing_amd import Scene, WavefrontPathTracer
    monkeypatch.setenv("DCRT_NO_LDS_CACHE", "1")
    monkeypatch.setenv("DCRT_PAIR_TRAVERSAL", "1")
    if scene_name == "cornell":
        s = cornell(48, 40, 6)
    else:
        s = Scene((32, 32))
        s.load_from_file(GOLDEN / "xml_mix" / "scene.xml")
    t = WavefrontPathTracer(path_pool_size=1 << 14, debug_rng=True)
    try:
        t.set_luts(golden_luts)
        t.on_scene_loaded(s)
        assert t.info()["pair_traversal"] == 1
        flat = oracle_mod.flat_with_own_bvh(s)
        for features in (0x0D, 0x07):
            rays = _rays(20000, 5 + features, scene_name == "cornell")
            assert np.array_equal(t.trace_rays(rays, features).view(np.uint8), oracle_mod.trace_rays(flat, rays, features)[0].view(np.uint8))
            assert np.array_equal(t.occluded(rays, features), oracle_mod.occluded(flat, rays, features)[0])
        t.set_mode("megakernel")
        t.clear_film()
        t.render_images(4, 1)
        pos, val = t.read_samples()
        p_ref, v_ref, r_ref, _ = oracle_mod.render(flat, golden_luts, oracle_mod.frame_params(s, 4), oracle_mod.MEGAKERNEL, rng=True)
        assert np.array_equal(t.read_rng(), r_ref)
        assert np.array_equal(pos.view(np.uint32), p_ref.view(np.uint32))
        assert same_bits(val, v_ref).all()
    finally:
        t.destroy()


@pytest.mark.parametrize("name", ["mask_xml", "spaceship"])
def test_pair_order_wavefront_anyhit_and_instancing_bit_exact(native_lib, golden_luts, oracle_mod, monkeypatch, name):
    """The pair kernels on the child-pair order, forced on small scenes: the any-hit shader's
    variant (mask_xml, ALLOW_ANYHIT_SHADER) and a BLAS shared by several instances (the
    spaceship fixture: four ships, one hull BLAS)."""
    from directcomputeraytracing_amd import WavefrontPathTracer
    from test_oracle import load_fixture_scene
    monkeypatch.setenv("DCRT_NO_LDS_CACHE", "1")
    monkeypatch.setenv("DCRT_PAIR_TRAVERSAL", "1")
    s = _anyhit_scenes()["mask_xml"] if name == "mask_xml" else load_fixture_scene("spaceship")
    t = WavefrontPathTracer(path_pool_size=1 << 14, debug_rng=True)
    try:
        list(_render_and_compare(t, oracle_mod, golden_luts, s, [0, 2]))
        assert t.info()["pair_traversal"] == 1
    finally:
        t.destroy()


def test_cpp_host_example_matches_python_host(native_lib, tmp_path):
    """examples/dcrt_render (C++ host over the C ABI, the reference's frame loop: Render /
    IsImageComplete / SampleConvolution per image) and its --batch mode (render_images)
    write the same BMP as the Python host's render_images + resolve_image."""
    import subprocess
    from directcomputeraytracing_amd import WavefrontPathTracer, save_bmp, scenes
    from directcomputeraytracing_amd.build import build_examples
    exe = build_examples()
    W, H, spp, bounces = 96, 64, 3, 4
    px, col = scenes.POINT_LIGHT_POSITION, scenes.POINT_LIGHT_COLOR
    light = ["--point", *map(str, px), *map(str, col)]
    out = {}
    for mode in ("frame", "batch"):
        bmp = tmp_path / f"{mode}.bmp"
        args = [str(exe), str(scenes.CORNELL_OBJ), str(W), str(H), str(spp), str(bounces), str(bmp), *light]
        r = subprocess.run(args + (["--batch"] if mode == "batch" else []), capture_output=True, text=True, timeout=300)
        assert r.returncode == 0, r.stderr
        out[mode] = bmp.read_bytes()
    s = cornell(W, H, bounces)
    t = WavefrontPathTracer(path_pool_size=1 << 16)
    try:
        t.on_scene_loaded(s)
        t.clear_film()
        t.render_images(0, spp)
        save_bmp(tmp_path / "py.bmp", t.resolve_image(s.postfx_params()))
    finally:
        t.destroy()
    assert out["frame"] == out["batch"] == (tmp_path / "py.bmp").read_bytes()


def _run_frame_loop(exe, tmp_path, tag, W, H, spp, bounces, *extra):
    import json
    import subprocess
    from directcomputeraytracing_amd import scenes
    px, col = scenes.POINT_LIGHT_POSITION, scenes.POINT_LIGHT_COLOR
    film, samples = tmp_path / f"{tag}.film", tmp_path / f"{tag}.samples"
    args = [str(exe), str(scenes.CORNELL_OBJ), str(W), str(H), str(spp), str(bounces), str(tmp_path / f"{tag}.bmp"),
            "--point", *map(str, px), *map(str, col), "--pool", str(1 << 16), "--film", str(film), "--samples", str(samples),
            *extra]
    r = subprocess.run(args, capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr
    info = json.loads(r.stdout.strip().splitlines()[-1])
    n = W * H
    raw = np.fromfile(samples, np.float32)
    return info, np.fromfile(film, np.float32).reshape(H, W, 4), raw[:2 * n].reshape(H, W, 2), raw[2 * n:].reshape(H, W, 4)


@pytest.mark.parametrize("policy", ["sample-count", "frame-index", "fixed"])
def test_cpathtracer_frame_loop_seed_policies(native_lib, tmp_path, policy):
    """CMI355XPathTracer (examples/mi355x_path_tracer.h: the reference's eight-virtual CPathTracer
    slot, PathTracer.h:6-26, over the C ABI alone) driven by the reference's frame loop
    (examples/renderer_loop.h: LaunchRendererLoop.cpp:159-298). The first frame after the load is
    the film-dirty quarter-resolution preview (:206-213, :405-406), convolved and then cleared by
    the resolution change; the frame seed is CScene::m_FrameSeed (WavefrontPathTracer.cpp:412)
    under each EFrameSeedType policy (:229-264); SampleConvolution runs once per completed image
    (:295-297). With 3 iterations per frame an image spans several Render calls.
      * SampleCount: the film of the spp images is render_images(0, spp)'s, bit for bit;
      * FrameIndex: the seed is not reset after the preview, so the images are first_seed ..;
      * Fixed (seed 5): every image repeats seed 5's samples; the film is render_images(5, 1)
        convolved spp times."""
    from directcomputeraytracing_amd import WavefrontPathTracer
    from directcomputeraytracing_amd.build import build_examples
    exe = build_examples()
    W, H, spp, bounces = 96, 64, 3, 4
    # (FrameIndex: 16 iterations per frame, so the 24 x 16 preview image completes in its frame)
    extra = ["--seed-type", policy, "--iterations", "16" if policy == "frame-index" else "3"]
    if policy == "fixed":
        extra += ["--fixed-seed", "5"]
    info, film, pos, val = _run_frame_loop(exe, tmp_path, policy, W, H, spp, bounces, *extra)
    assert info["mode"] == "frame_loop" and info["preview_frames"] == 1 and info["images"] == spp
    s = cornell(W, H, bounces)
    t = WavefrontPathTracer(path_pool_size=1 << 16)
    try:
        t.on_scene_loaded(s)
        t.clear_film()
        if policy == "sample-count":
            assert info["seeds"] == list(range(spp))
            t.render_images(0, spp)
        elif policy == "frame-index":
            # the preview completed its image at seed 0 and advanced the seed; FrameIndex does
            # not reset it, so the full-resolution images are seeds 1 ..
            first = info["first_seed"]
            assert first == 1 and info["seeds"] == list(range(first, first + spp))
            t.render_images(first, spp)
        else:
            assert info["seeds"] == [5] * spp
            t.render_images(5, 1)
            for _ in range(spp - 1):
                t.accumulate_film()
        ref_pos, ref_val = t.read_samples()
        ref_film = t.read_film()
    finally:
        t.destroy()
    assert same_bits(pos, ref_pos).all() and same_bits(val, ref_val).all()
    assert same_bits(film, ref_film).all()


def test_postfx_resolve_bit_exact(native_lib, golden_luts, oracle_mod):
    """Exposure (manual / auto via the two-stage log-luminance reduction) + Reinhard + sRGB8."""
    from directcomputeraytracing_amd import PostFxParams, WavefrontPathTracer, srgb_thresholds
    t = WavefrontPathTracer(path_pool_size=1 << 16)
    try:
        s = cornell(100, 70, 3)
        t.set_luts(golden_luts)
        t.on_scene_loaded(s)
        t.clear_film()
        t.render_images(0, 2)
        film = t.read_film()
        th = srgb_thresholds()
        for prm in (PostFxParams(1, 1, 0.0, 1.0), PostFxParams(1, 0, s.postfx_params().ev100, 2.0),
                    PostFxParams(0, 0, 0.0, 1.0)):
            img, lum = t.resolve_image(prm, with_luminance=True)
            ref = oracle_mod.resolve_image(film, prm, th)
            assert np.array_equal(img, ref)
        assert same_bits(np.float32(lum), np.float32(oracle_mod.sum_log_luminance(film)))
    finally:
        t.destroy()


@pytest.mark.parametrize("scene_name", ["cornell", "xml_mix", "lamp"])
def test_megakernel_matches_oracle_megakernel(native_lib, golden_luts, oracle_mod, scene_name):
    """CMegakernelPathTracer on the GPU == the oracle's MegakernelPathTracing restatement,
    including bounce-0 triangle emission (where it differs from the wavefront, Appendix A.6)."""
    from conftest import GOLDEN
    from directcomputeraytracing_amd import Scene, WavefrontPathTracer
    if scene_name == "cornell":
        s = cornell(96, 72, 6)
    elif scene_name == "xml_mix":
        s = Scene((8, 8))
        s.load_from_file(GOLDEN / "xml_mix" / "scene.xml")
    else:
        from test_oracle import load_fixture_scene
        s = load_fixture_scene("lamp")
    t = WavefrontPathTracer(path_pool_size=1 << 15, debug_rng=True)
    try:
        t.set_luts(golden_luts)
        t.on_scene_loaded(s)
        t.set_mode("megakernel")
        for seed in (0, 3):
            t.clear_film()
            t.render_images(seed, 1)
            pos, val = t.read_samples()
            rng = t.read_rng()
            p_ref, v_ref, r_ref, c_ref = oracle_mod.render(oracle_mod.flat_with_own_bvh(s), golden_luts, oracle_mod.frame_params(s, seed), oracle_mod.MEGAKERNEL,
                                                           rng=True)
            assert np.array_equal(rng, r_ref)
            assert np.array_equal(pos.view(np.uint32), p_ref.view(np.uint32))
            bad = np.count_nonzero(~same_bits(val, v_ref).all(-1))
            assert bad == 0, f"{scene_name} seed {seed}: {bad} pixels differ"
    finally:
        t.destroy()


def test_megakernel_full_size_cornell_bit_exact(native_lib, golden_luts, oracle_mod):
    """The megakernel mode (bench.py --mode megakernel) at the headline size: Cornell 1920x1080,
    8 bounces, the bench's default pool, image 0 -- every sample and the ray counts equal the
    oracle's MegakernelPathTracing restatement."""
    from directcomputeraytracing_amd import WavefrontPathTracer, scenes
    s = cornell(1920, 1080, 8)
    t = WavefrontPathTracer(path_pool_size=scenes.default_pool(1920, 1080))
    try:
        t.set_luts(golden_luts)
        t.on_scene_loaded(s)
        t.set_mode("megakernel")
        t.reset_stats()
        t.render_images(0, 1)
        pos, val = t.read_samples()
        c = t.counters()
    finally:
        t.destroy()
    p_ref, v_ref, _, c_ref = oracle_mod.render(oracle_mod.flat_with_own_bvh(s), golden_luts, oracle_mod.frame_params(s, 0),
                                               oracle_mod.MEGAKERNEL)
    assert np.array_equal(pos.view(np.uint32), p_ref.view(np.uint32))
    bad = np.count_nonzero(~same_bits(val, v_ref).all(-1))
    assert bad == 0, f"{bad} of {val.shape[0] * val.shape[1]} pixels differ"
    assert (c["extension_rays"], c["shadow_rays"]) == (c_ref["extension_rays"], c_ref["shadow_rays"]), (c, c_ref)


# ---- ALLOW_ANYHIT_SHADER ------------------------------------------------------------------
def _anyhit_scenes():
    from directcomputeraytracing_amd import FEATURE_ALLOW_ANYHIT
    from test_oracle import anyhit_scene
    s = anyhit_scene()
    s.features = s.features | FEATURE_ALLOW_ANYHIT
    c = cornell(48, 40, 6)
    c.features = c.features | FEATURE_ALLOW_ANYHIT
    c.set_material_opacity(3, 0.5, -1)          # short box: per-triangle material ids, no override
    c.set_material_opacity(4, 0.25, -1)
    return {"mask_xml": s, "cornell_translucent": c}


@pytest.mark.parametrize("name", ["mask_xml", "cornell_translucent"])
def test_anyhit_wavefront_bit_exact(gpu_tracer, golden_luts, oracle_mod, name):
    """Opacity samples drawn by NEW_PATH / MATERIAL (:223-226, :422-430), the AnyHitShader
    with float and bitmap opacity, OBJ material ids and rectangle instance overrides."""
    s = _anyhit_scenes()[name]
    list(_render_and_compare(gpu_tracer, oracle_mod, golden_luts, s, [0, 5]))


@pytest.mark.parametrize("name", ["mask_xml", "cornell_translucent"])
def test_anyhit_megakernel_bit_exact(native_lib, golden_luts, oracle_mod, name):
    """MegakernelPathTracing.hlsl draws the opacity samples inside IntersectScene/IsOcculuded."""
    from directcomputeraytracing_amd import WavefrontPathTracer
    s = _anyhit_scenes()[name]
    t = WavefrontPathTracer(path_pool_size=1 << 15, debug_rng=True)
    try:
        t.set_luts(golden_luts)
        t.on_scene_loaded(s)
        t.set_mode("megakernel")
        t.clear_film()
        t.render_images(2, 1)
        pos, val = t.read_samples()
        p_ref, v_ref, r_ref, _ = oracle_mod.render(oracle_mod.flat_with_own_bvh(s), golden_luts, oracle_mod.frame_params(s, 2), oracle_mod.MEGAKERNEL, rng=True)
        assert np.array_equal(t.read_rng(), r_ref)
        assert np.array_equal(pos.view(np.uint32), p_ref.view(np.uint32))
        assert same_bits(val, v_ref).all()
    finally:
        t.destroy()


# (cornell-20: the driver's timed configuration, bench.py --steps 20 -- one 20-image batch per pipeline)
@pytest.mark.parametrize("config,images", [("cornell", 4), ("cornell", 20), ("coffee", 1), ("spaceship", 1),
                                           ("spaceship_close", 1), ("lamp", 1)])
def test_bench_configuration_full_size_bit_exact(native_lib, golden_luts, oracle_mod, tmp_path, config, images):
    """The bench's own configurations at full size, built by the bench's own code
    (make_pipelines, as bench.py does): 8 bounces (lamp: its XML's depth), the default pool (2^24
    slots per pipeline at 1080p, 2^26 at 4K) split over the bench's concurrent stream-partitioned
    pipelines (three for Cornell, two elsewhere), virtual
    batch starts, the GPU-built LUTs and each config's default cast kernel -- Cornell 1080p: the
    cache-only IDENT kernel; coffee 1080p (configs[2], Kulla-Conty on): the global-memory kernel;
    spaceship 4K (configs[3], the 522 k-node hull x 8, wide and close framing): the pair kernel
    with the LDS stack ring;
    lamp 4K (configs[4], thin lens, triangle lights). Images 0..N-1 rendered concurrently, the two
    films summed on the device. The combined film must equal the oracle's film of the same images
    bit for bit, and the ray counts the oracle's (plus the halo rows both pipelines trace)."""
    from directcomputeraytracing_amd import Scene, make_pipelines, probe_row_cost, render_images_concurrently, scenes
    s = Scene((1920, 1080))
    if config == "cornell":
        scenes.setup_cornell(s, 1920, 1080, 8)
    elif config == "coffee":
        scenes.setup_config(s, "coffee", str(tmp_path), multiscattering=True)
    else:
        scenes.setup_config(s, config, str(tmp_path))
    W, H = s.resolution
    assert (W, H) == ((3840, 2160) if config in ("spaceship", "spaceship_close", "lamp") else (1920, 1080))
    filt = s.filter_params()
    K = 3 if config == "cornell" else 2   # (bench.py's default pipelines per GPU)
    # bench.py's default film tiling: cost-balanced bands from the row-cost probe
    cost = probe_row_cost(s)
    ts = make_pipelines(s, scenes.default_pool(W, H, K), streams=K, images=images, iterations=16, row_cost=cost)
    try:
        info = ts[0].info()
        if config == "cornell":
            assert info["scene_in_lds"] == 1 and info["cast_identity"] == 2   # (IDENT over the entry-free order)
        elif config == "coffee":
            assert info["scene_in_lds"] == 0 and info["pair_traversal"] == 0
        elif config.startswith("spaceship"):
            assert info["pair_traversal"] == 1 and info["ring_rows"] == 16
        for t in ts:
            t.clear_film()
            t.reset_stats()
        render_images_concurrently(ts, 0, images, filt)
        for t in ts[1:]:
            ts[0].add_film_device(t.film_device_ptr())
        ts[0].synchronize()
        film = ts[0].read_film()
        ext = sum(t.counters()["extension_rays"] for t in ts)
        shadow = sum(t.counters()["shadow_rays"] for t in ts)
    finally:
        for t in ts:
            t.destroy()
    flat = oracle_mod.flat_with_own_bvh(s)
    ref = np.zeros_like(film)
    ext_ref = shadow_ref = 0
    # the rows two pipelines path-trace (each renders the filter's halo rows beyond its band):
    # their rays are traced twice
    from directcomputeraytracing_amd.partition import balanced_bands, band_render_rows, halo_for_radius
    halo = max(1, halo_for_radius(filt.radius, H))
    times = np.zeros(H, np.int64)
    for band in balanced_bands(cost, K, halo):
        times[band_render_rows(H, [band], halo)] += 1
    assert (times >= 1).all() and times.max() <= 2
    twice = sorted(np.nonzero(times == 2)[0].tolist())
    assert 0 < len(twice) <= 4 * halo * (K - 1)
    for seed in range(images):
        fr = oracle_mod.frame_params(s, seed)
        p, v, _, c = oracle_mod.render(flat, golden_luts, fr, oracle_mod.WAVEFRONT)
        oracle_mod.sample_convolution(filt, p, v, ref)
        ext_ref += c["extension_rays"]
        shadow_ref += c["shadow_rays"]
        for y in twice:
            _, _, _, c = oracle_mod.render(flat, golden_luts, fr, oracle_mod.WAVEFRONT, rect=(0, y, W, 1))
            ext_ref += c["extension_rays"]
            shadow_ref += c["shadow_rays"]
    bad = np.count_nonzero(~same_bits(film, ref).all(-1))
    assert bad == 0, f"{bad} film pixels differ"
    assert (ext, shadow) == (ext_ref, shadow_ref)


def test_rank_share_full_size_bit_exact(native_lib, golden_luts, oracle_mod):
    """One rank's share of the N = 8 Cornell bench exactly as bench.py builds it on that rank
    (make_pipelines: world 8, rank 3, three image-interleaved pipelines over the rank's one
    cost-balanced band, cut from the row-cost probe after a calibration re-cut by rank times --
    here a synthetic 8 % trend down the image), images 0-2 at 1920x1080 / 8 bounces (one per
    pipeline): the rank's film equals the oracle's film on the rows it owns, convolved in image
    order, and is zero elsewhere; its ray counts are the oracle's over the rows it path-traces
    (owned rows plus the filter's halo)."""
    from directcomputeraytracing_amd import (Scene, make_pipelines, prepare_pipelines, probe_row_cost,
                                             render_images_concurrently, scenes)
    from directcomputeraytracing_amd.partition import (balanced_bands, band_owned_rows, band_render_rows, halo_for_radius,
                                                       refine_row_cost, row_runs)
    W, H, world, rank, K, images = 1920, 1080, 8, 3, 3, 3
    s = Scene((W, H))
    scenes.setup_cornell(s, W, H, 8)
    filt = s.filter_params()
    halo = max(1, halo_for_radius(filt.radius, H))
    probe = probe_row_cost(s)
    first = balanced_bands(probe, world, halo)
    cost = refine_row_cost(probe, [[b] for b in first], [1.0 + 0.01 * r for r in range(world)], halo)
    ts = make_pipelines(s, scenes.default_pool(W, H, K), streams=K, images=images, iterations=16, world=world, rank=rank,
                        row_cost=cost, interleave=True, bands_per_rank=1)
    try:
        prepare_pipelines(ts, images)
        for t in ts:
            t.clear_film()
            t.reset_stats()
        render_images_concurrently(ts, 0, images, filt)
        ts[0].synchronize()
        film = ts[0].read_film()
        assert all(not t.read_film().any() for t in ts[1:])
        ext = sum(t.counters()["extension_rays"] for t in ts)
        shadow = sum(t.counters()["shadow_rays"] for t in ts)
    finally:
        for t in ts:
            t.destroy()
    mine = balanced_bands(cost, world, halo)[rank::world]
    assert len(mine) == 1 and mine != [first[rank]], "the calibrated cut is not the probe's"
    owned = band_owned_rows(H, mine)
    assert 0 < owned.sum() < H // 4
    flat = oracle_mod.flat_with_own_bvh(s)
    ref = np.zeros_like(film)
    ext_ref = shadow_ref = 0
    for image in range(images):
        fr = oracle_mod.frame_params(s, image)
        pos = np.zeros((H, W, 2), np.float32)
        val = np.zeros((H, W, 4), np.float32)
        for y0, y1 in row_runs(band_render_rows(H, mine, halo)):
            p, v, _, c = oracle_mod.render(flat, golden_luts, fr, oracle_mod.WAVEFRONT, rect=(0, y0, W, y1 - y0))
            pos[y0:y1], val[y0:y1] = p[y0:y1], v[y0:y1]
            ext_ref += c["extension_rays"]
            shadow_ref += c["shadow_rays"]
        for y0, y1 in row_runs(np.nonzero(owned)[0]):
            oracle_mod.sample_convolution(filt, pos, val, ref, rows=(y0, y1))
    assert not film[~owned].any(), "the rank wrote rows it does not own"
    bad = np.count_nonzero(~same_bits(film[owned], ref[owned]).all(-1))
    assert bad == 0, f"{bad} owned film pixels differ"
    assert (ext, shadow) == (ext_ref, shadow_ref)


KNOB_CASES = [
    # (id, scene, env): scheduling / sizing knobs of dcrt_tracer::UploadScene and persistent_trace
    ("block64_global", "xml_mix", {"DCRT_CAST_BLOCK": "64", "DCRT_NO_LDS_CACHE": "1"}),
    ("block128_pair", "xml_mix", {"DCRT_CAST_BLOCK": "128", "DCRT_NO_LDS_CACHE": "1", "DCRT_PAIR_TRAVERSAL": "1"}),
    ("blocks_per_cu_2", "lamp", {"DCRT_CAST_BLOCKS_PER_CU": "2"}),
    ("grid_mul_3", "lamp", {"DCRT_CAST_GRID_MUL": "3"}),
    ("lds_reserve_0_no_trim", "lamp", {"DCRT_CAST_LDS_RESERVE": "0", "DCRT_LDS_TRIM": "0"}),
    ("material_lds_not_partial", "lamp", {"DCRT_MATERIAL_LDS_PARTIAL": "0"}),
    ("top_nodes_64", "spaceship", {"DCRT_PAIR_TRAVERSAL": "1", "DCRT_TOP_NODES": "64"}),
    ("tune_8_4", "cornell", {"DCRT_TRAVERSAL_TUNE": "8,4"}),
    ("tune_64_64", "cornell", {"DCRT_TRAVERSAL_TUNE": "64,64", "DCRT_NO_LDS_CACHE": "1"}),
    # trav_skip_root: off, and 16 levels of sure hits (cache-only, entry-free order / global-memory kernel)
    ("skip_root_off", "cornell", {"DCRT_SKIP_ROOT": "0"}),
    ("skip_root_16", "cornell", {"DCRT_SKIP_ROOT": "16"}),
    ("skip_root_16_global", "xml_mix", {"DCRT_SKIP_ROOT": "16", "DCRT_PAIR_TRAVERSAL": "0"}),
    ("flat_cast_off", "cornell", {"DCRT_FLAT_CAST": "0"}),
    ("flat_no_merge", "cornell", {"DCRT_FLAT_MERGE": "0"}),
]


@pytest.mark.parametrize("case,scene_name,env", KNOB_CASES, ids=[c[0] for c in KNOB_CASES])
def test_tuning_knobs_bit_exact(native_lib, golden_luts, oracle_mod, monkeypatch, case, scene_name, env):
    """Every A/B knob the tracer reads (workgroup size, resident workgroups per CU, grid multiple,
    the LDS cache's reserve and trim, MATERIAL's partial LDS copy, the pair order's breadth-first
    prefix, the refill / park thresholds) changes scheduling or sizing only: the wavefront render
    stays bit-exact against the oracle."""
    from conftest import GOLDEN
    from directcomputeraytracing_amd import Scene, WavefrontPathTracer
    from test_oracle import load_fixture_scene
    for k, v in env.items():
        monkeypatch.setenv(k, v)
    if scene_name == "cornell":
        s = cornell(64, 48, 6)
    elif scene_name == "xml_mix":
        s = Scene((32, 32))
        s.load_from_file(GOLDEN / "xml_mix" / "scene.xml")
    else:
        s = load_fixture_scene(scene_name)
    t = WavefrontPathTracer(path_pool_size=1 << 14, debug_rng=True)
    try:
        list(_render_and_compare(t, oracle_mod, golden_luts, s, [0, 3]))
        info = t.info()
        if "DCRT_CAST_BLOCK" in env:
            assert info["cast_block"] == int(env["DCRT_CAST_BLOCK"])
        if "DCRT_CAST_BLOCKS_PER_CU" in env:
            assert info["cast_grid"] == 2 * 256
    finally:
        t.destroy()
