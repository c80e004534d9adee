"""Seeded random scenes (tests/random_scenes.py): triangle soups with shared edges, flat patches,
zero-area and coincident triangles, transformed and identity instances, every BSDF type and light
kind, pinhole and thin-lens cameras.

CPU: the product's XML translation equals the oracle's restatement over the reference's own
RapidXml / tinyobjloader / MikkTSpace (where oracle/_ref is built), and the product's flattened
scene (BVH build included) equals the oracle's own flattening, array for array, bit for bit.
GPU: every cast kernel variant the tracer can pick for such a scene -- the LDS-cached one (the
cache-only IDENT kernel for the OBJ scenes), the global-memory one, the pair traversal and the
8-row stack ring that spills, the opacity kernels, the split EXT / SHADOW casts, CONTROL-written
batch starts and the drain-completion kernel -- and the megakernel render the oracle's image bit
for bit."""
import os

import numpy as np
import pytest

import random_scenes as R
from test_xml_translation_pin import REFOBJ, REFXML, check, oracle_xml  # noqa: F401 (oracle_xml: a fixture)

SEEDS = range(int(os.environ.get("DCRT_RANDOM_SCENE_SEEDS", "6")))   # (more for a soak run)


def _scene(kind, seed, tmp_path):
    from directcomputeraytracing_amd import Scene
    s = Scene((48, 36))
    if kind == "obj":
        R.setup_obj_scene(s, R.write_obj_scene(tmp_path, seed), seed)
    else:
        s.load_from_file(R.write_xml_scene(tmp_path, seed))
    return s


@pytest.mark.parametrize("seed", SEEDS)
@pytest.mark.skipif(not (REFXML.exists() and REFOBJ.exists()), reason="oracle/_ref reference checkers not built (no /root/reference)")
def test_random_xml_translation_matches_oracle(oracle_xml, seed, tmp_path):
    o = check(oracle_xml, R.write_xml_scene(tmp_path, seed))
    assert o is not None and len(o["instances"]) >= 4


@pytest.mark.parametrize("kind", ["obj", "xml"])
@pytest.mark.parametrize("seed", SEEDS)
def test_random_scene_flattening_matches_oracle(native_lib, oracle_mod, tmp_path, kind, seed):
    from test_scene_pin import _flat_arrays
    s = _scene(kind, seed, tmp_path)
    prod = _flat_arrays(s.flat())
    own = _flat_arrays(oracle_mod.flatten_scene(s))
    for k in prod:
        assert prod[k].shape == own[k].shape and np.array_equal(prod[k], own[k]), (kind, seed, k)
    a, b = s.frame_params(seed), oracle_mod.frame_params(s, seed)
    assert bytes(a) == bytes(b)


@pytest.mark.gpu
@pytest.mark.parametrize("cache", ["lds", "global", "pair", "ring8", "megakernel", "anyhit", "split", "no_virtual", "drain"])
@pytest.mark.parametrize("kind", ["obj", "xml"])
@pytest.mark.parametrize("seed", SEEDS)
def test_random_scenes_bit_exact(native_lib, golden_luts, oracle_mod, monkeypatch, tmp_path, kind, seed, cache):
    from test_gpu_parity import _render_and_compare, same_bits
    from directcomputeraytracing_amd import WavefrontPathTracer
    if cache in ("global", "pair"):
        monkeypatch.setenv("DCRT_NO_LDS_CACHE", "1")
    monkeypatch.setenv("DCRT_PAIR_TRAVERSAL", "1" if cache == "pair" else "0")
    if cache == "ring8":
        monkeypatch.setenv("DCRT_NO_LDS_CACHE", "1")
        monkeypatch.setenv("DCRT_STACK_RING", "8")
    # the reference's two cast kernels (EXT, then SHADOW), batch starts written out by CONTROL,
    # and the drain-completion kernel for the last few hundred paths
    if cache == "split":
        monkeypatch.setenv("DCRT_SPLIT_CASTS", "1")
    if cache == "no_virtual":
        monkeypatch.setenv("DCRT_VIRTUAL_START", "0")
    if cache == "drain":
        monkeypatch.setenv("DCRT_DRAIN_PATHS", "300")
    s = _scene(kind, seed, tmp_path)
    if cache == "anyhit":   # ALLOW_ANYHIT_SHADER with translucent materials: the OPACITY kernels
        rng = np.random.default_rng(seed + 77)
        s.features = s.features | 0x10
        for i in range(s.material_count):
            if rng.random() < 0.6:
                s.set_material_opacity(i, float(rng.uniform(0.2, 0.9)))
    t = WavefrontPathTracer(path_pool_size=1 << 12, debug_rng=True)
    try:
        if cache == "megakernel":
            t.set_luts(golden_luts)
            t.on_scene_loaded(s)
            t.set_mode("megakernel")
            for fs in (0, 5):
                t.clear_film()
                t.render_images(fs, 1)
                pos, val = t.read_samples()
                p_ref, v_ref, _, _ = oracle_mod.render(oracle_mod.flat_with_own_bvh(s), golden_luts, oracle_mod.frame_params(s, fs),
                                                       oracle_mod.MEGAKERNEL)
                assert np.array_equal(pos.view(np.uint32), p_ref.view(np.uint32))
                bad = np.count_nonzero(~same_bits(val, v_ref).all(-1))
                assert bad == 0, f"{kind} seed {seed} frame {fs}: {bad} pixels differ"
            return
        rays = [0, 0]
        for c, c_ref in _render_and_compare(t, oracle_mod, golden_luts, s, [0, 5]):
            rays = [rays[0] + c_ref["extension_rays"], rays[1] + c_ref["shadow_rays"]]   # (the tracer's counts accumulate)
            assert [c["extension_rays"], c["shadow_rays"]] == rays
        info = t.info()
        assert info["pair_traversal"] == (1 if cache == "pair" else 0)
        if cache == "lds" and kind == "obj":   # (the XML scenes' soup is partly cached: nodes in LDS, the rest global)
            assert info["scene_in_lds"] == 1 and info["cast_identity"] in (1, 2)
        if cache == "ring8":
            assert info["ring_rows"] == 8
    finally:
        t.destroy()


def _aimed_rays(flat_arrays, seed, n_origins=24):
    """Rays aimed at the scene's vertices and edge midpoints as every instance places them (exact
    vertex / shared-edge hits: several triangles at one distance), from random origins and from
    the vertices themselves (tMin = 0 on the surface), plus axis-aligned rays through vertices."""
    from directcomputeraytracing_amd import make_rays
    rng = np.random.default_rng(seed)
    pos = flat_arrays["vertices"][:, :3].view(np.float32).astype(np.float64)
    tri = flat_arrays["triangles"].astype(np.int64)
    mids = 0.5 * (pos[tri[:, 0]] + pos[tri[:, 1]])
    pts = np.concatenate([pos, mids])
    xf = flat_arrays["instance_transforms"].view(np.float32).astype(np.float64)
    n_inst = len(xf) // 2
    world = np.concatenate([np.c_[pts, np.ones(len(pts))] @ xf[i].reshape(4, 3) for i in range(n_inst)])
    world = world[rng.choice(len(world), min(len(world), 4000), replace=False)]
    o = rng.uniform([-3, -0.2, -5], [3, 3, 3], (n_origins, 3))
    above = world + np.array([0.0, 2.0, 0.0])
    O = np.concatenate([np.repeat(o, len(world), 0), world, above])
    T = np.concatenate([np.tile(world, (n_origins, 1)), world[rng.permutation(len(world))], world])
    D = T - O                                      # (the last block: straight down through every vertex)
    keep = np.linalg.norm(D, axis=1) > 1e-9
    O, D = O[keep], D[keep]
    D /= np.linalg.norm(D, axis=1, keepdims=True)
    r = make_rays(O.astype(np.float32), D.astype(np.float32), 0.0, np.inf)
    k = len(r) // 4
    r["t_max"][:k] = rng.uniform(0.05, 3.0, k)
    return r


@pytest.mark.gpu
@pytest.mark.parametrize("features", [0x0D, 0x05])
@pytest.mark.parametrize("kind", ["obj", "xml"])
@pytest.mark.parametrize("seed", SEEDS)
def test_random_scene_aimed_rays_bit_exact(gpu_tracer, oracle_mod, tmp_path, kind, seed, features):
    """trace_rays / occluded (the closest-hit and any-hit casts) on rays aimed exactly at
    vertices and shared edges: hits, distances, barycentrics, triangle and instance ids and the
    occlusion bits equal the oracle's (its visit order settles every tie)."""
    from test_scene_pin import _flat_arrays
    s = _scene(kind, seed, tmp_path)
    gpu_tracer.on_scene_loaded(s)
    flat = oracle_mod.flat_with_own_bvh(s)
    rays = _aimed_rays(_flat_arrays(flat), seed)
    assert len(rays) > 10000
    h_gpu = gpu_tracer.trace_rays(rays, features)
    h_cpu, _ = oracle_mod.trace_rays(flat, rays, features)
    bad = np.nonzero((h_gpu.view(np.uint8).reshape(len(rays), -1) != h_cpu.view(np.uint8).reshape(len(rays), -1)).any(1))[0]
    assert len(bad) == 0, f"{len(bad)} of {len(rays)} hits differ, first {bad[:5]}"
    assert np.array_equal(gpu_tracer.occluded(rays, features), oracle_mod.occluded(flat, rays, features)[0])
    hit = np.isfinite(h_cpu["t"]) if "t" in (h_cpu.dtype.names or ()) else None
    if hit is not None:
        assert hit.mean() > 0.05   # (the rays do reach the geometry)


@pytest.mark.gpu
@pytest.mark.parametrize("kind", ["obj", "xml"])
@pytest.mark.parametrize("seed", SEEDS)
def test_random_scene_pipelines_bit_exact(native_lib, golden_luts, oracle_mod, tmp_path, kind, seed):
    """The bench's construction (make_pipelines: two stream-partitioned pipelines with halo rows,
    virtual batch starts, image batches) on a random scene, 64x160 so both pipelines own
    stripes: the device-summed film of images 0..2 equals the oracle's film, and the ray counts
    its counts (halo rows traced by both pipelines counted twice)."""
    from test_gpu_parity import same_bits
    from directcomputeraytracing_amd import Scene, make_pipelines, render_images_concurrently
    from directcomputeraytracing_amd.partition import halo_for_radius, render_rows, stream_partition
    W, H, images = 64, 160, 3
    s = Scene((W, H))
    if kind == "obj":
        R.setup_obj_scene(s, R.write_obj_scene(tmp_path, seed), seed, W, H)
    else:
        s.load_from_file(R.write_xml_scene(tmp_path, seed, W, H))
    assert tuple(s.resolution) == (W, H)
    filt = s.filter_params()
    ts = make_pipelines(s, 1 << 12, streams=2, images=images, iterations=8)
    try:
        for t in ts:   # (the tracers' own GPU-built LUTs: bit-identical to the golden ones)
            t.clear_film()
            t.reset_stats()
        render_images_concurrently(ts, 0, images, filt)
        ts[0].add_film_device(ts[1].film_device_ptr())
        ts[0].synchronize()
        film = ts[0].read_film()
        ext = sum(t.counters()["extension_rays"] for t in ts)
        shadow = sum(t.counters()["shadow_rays"] for t in ts)
    finally:
        for t in ts:
            t.destroy()
    flat = oracle_mod.flat_with_own_bvh(s)
    ref = np.zeros_like(film)
    halo = max(1, halo_for_radius(filt.radius, H))
    a, b = (set(render_rows(H, *stream_partition(H, 1, 0, 2, k, 64), halo)) for k in range(2))
    twice = sorted(a & b)
    ext_ref = shadow_ref = 0
    for fs in range(images):
        fr = oracle_mod.frame_params(s, fs)
        p, v, _, c = oracle_mod.render(flat, golden_luts, fr, oracle_mod.WAVEFRONT)
        oracle_mod.sample_convolution(filt, p, v, ref)
        ext_ref += c["extension_rays"]
        shadow_ref += c["shadow_rays"]
        for y in twice:
            _, _, _, c = oracle_mod.render(flat, golden_luts, fr, oracle_mod.WAVEFRONT, rect=(0, y, W, 1))
            ext_ref += c["extension_rays"]
            shadow_ref += c["shadow_rays"]
    bad = np.count_nonzero(~same_bits(film, ref).all(-1))
    assert bad == 0, f"{kind} seed {seed}: {bad} film pixels differ"
    assert (ext, shadow) == (ext_ref, shadow_ref)


@pytest.mark.gpu
@pytest.mark.parametrize("cache", ["default", "pair", "ring8", "many_instances"])
@pytest.mark.parametrize("seed", range(int(os.environ.get("DCRT_RANDOM_LARGE_SEEDS", "2"))))
def test_random_large_scenes_bit_exact(native_lib, golden_luts, oracle_mod, monkeypatch, tmp_path, seed, cache):
    """A larger soup (a 48 x 48 height field + 600 loose triangles, about 5 k triangles per
    instance, 2-4 instances): deeper BVHs and stacks, the LDS node cache holding only the top of
    the tree, the pair traversal and a spilling 8-row ring on real depths; and a deep TLAS (24
    overlapping transformed instances of a small soup: many BLAS entries and exits per ray)."""
    from test_gpu_parity import _render_and_compare
    from directcomputeraytracing_amd import Scene, WavefrontPathTracer
    if cache != "default":
        monkeypatch.setenv("DCRT_PAIR_TRAVERSAL", "1" if cache == "pair" else "0")
    if cache == "ring8":
        monkeypatch.setenv("DCRT_STACK_RING", "8")
    s = Scene((48, 36))
    if cache == "many_instances":
        s.load_from_file(R.write_xml_scene(tmp_path, 2000 + seed, n_instances=24))
    else:
        s.load_from_file(R.write_xml_scene(tmp_path, 1000 + seed, n_grid=48, n_loose=600))
    t = WavefrontPathTracer(path_pool_size=1 << 12, debug_rng=True)
    try:
        rays = [0, 0]
        for c, c_ref in _render_and_compare(t, oracle_mod, golden_luts, s, [0, 5]):
            rays = [rays[0] + c_ref["extension_rays"], rays[1] + c_ref["shadow_rays"]]
            assert [c["extension_rays"], c["shadow_rays"]] == rays
        info = t.info()
        if cache == "many_instances":
            return
        assert info["scene_in_lds"] == 0 and info["traversal_stack"] >= 10, info
        assert info["pair_traversal"] == (1 if cache == "pair" else 0)
        if cache == "ring8":
            assert info["ring_rows"] == 8 and t.ring_spills() > 0
    finally:
        t.destroy()


@pytest.mark.gpu
@pytest.mark.parametrize("order", ["flat", "pairs"])
@pytest.mark.parametrize("kind", ["obj", "xml"])
@pytest.mark.parametrize("seed", SEEDS)
def test_random_scene_traversal_counters_match_oracle(native_lib, golden_luts, oracle_mod, monkeypatch, tmp_path, kind, seed,
                                                      order):
    """The counting cast kernels walk the reference's order node for node on random scenes too:
    node visits, triangle tests and BLAS entries of the extension and shadow rays equal the
    oracle's (BVHAccel.inc.hlsl's iterationCounter and friends), on PackBVH's node order and on the
    device's child-pair order."""
    from directcomputeraytracing_amd import WavefrontPathTracer
    if order == "pairs":
        monkeypatch.setenv("DCRT_NO_LDS_CACHE", "1")
        monkeypatch.setenv("DCRT_PAIR_TRAVERSAL", "1")
    s = _scene(kind, seed, tmp_path)
    t = WavefrontPathTracer(path_pool_size=1 << 12)
    try:
        t.set_luts(golden_luts)
        t.on_scene_loaded(s)
        assert t.info()["pair_traversal"] == (1 if order == "pairs" else 0)
        t.set_instrumentation(True, True)
        t.reset_stats()
        t.render_images(4, 1)
        st = t.traversal_stats()
        c = t.counters()
    finally:
        t.destroy()
    _, _, _, ref = oracle_mod.render(oracle_mod.flat_with_own_bvh(s), golden_luts, oracle_mod.frame_params(s, 4), oracle_mod.WAVEFRONT)
    assert (c["extension_rays"], c["shadow_rays"]) == (ref["extension_rays"], ref["shadow_rays"])
    got = [st[k] for k in ("ext_node_visits", "ext_triangle_tests", "ext_blas_entries", "shadow_node_visits",
                           "shadow_triangle_tests", "shadow_blas_entries")]
    want = [ref[k] for k in ("node_visits", "triangle_tests", "blas_entries", "shadow_node_visits", "shadow_triangle_tests",
                             "shadow_blas_entries")]
    assert got == want
