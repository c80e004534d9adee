"""GPU: the size limits of the path pool and the film sample arrays.

* Create() refuses a pool whose 64-B per-slot records would pass the 32-bit byte offsets
  the kernels address pool arrays with (2^26 slots is the largest accepted; the 4K bench
  uses exactly that), and a 2^26-slot pool renders a 3840-wide strip bit-exact against the
  oracle.
* A batch of more than 32 4K images puts the film sample arrays past 2^32 bytes
  (sample index x 16 B): the last image's samples must still land on their own pixels.
* UploadScene refuses a traversal stack size below the uploaded BVH's depth (the LDS
  stack pushes without a bound check).
"""
import numpy as np
import pytest

from conftest import cornell

pytestmark = pytest.mark.gpu


def same_bits(a, b):
    a, b = np.asarray(a, np.float32), np.asarray(b, np.float32)
    return (a.view(np.uint32) == b.view(np.uint32)) | (np.isnan(a) & np.isnan(b))


def test_create_refuses_pool_past_32bit_offsets(native_lib):
    from directcomputeraytracing_amd import DCRTError, WavefrontPathTracer
    with pytest.raises(DCRTError, match="LIMIT"):
        WavefrontPathTracer(path_pool_size=(1 << 26) + 256)


def test_2p26_pool_renders_4k_strip_bit_exact(native_lib, golden_luts, oracle_mod):
    from directcomputeraytracing_amd import WavefrontPathTracer
    t = WavefrontPathTracer(path_pool_size=1 << 26, iterations_per_render=16, debug_rng=True)
    try:
        s = cornell(3840, 24, 8)
        t.set_luts(golden_luts)
        t.on_scene_loaded(s)
        t.clear_film()
        t.render_images(11, 2)
        pos, val = t.read_samples()
        rng = t.read_rng()
        p_ref, v_ref, r_ref, _ = oracle_mod.render(oracle_mod.flat_with_own_bvh(s), golden_luts, oracle_mod.frame_params(s, 12),
                                                   oracle_mod.WAVEFRONT, rng=True)
        assert np.array_equal(rng, r_ref)
        assert same_bits(pos, p_ref).all() and same_bits(val, v_ref).all()
    finally:
        t.destroy()


def test_4k_batch_past_2p32_sample_bytes(native_lib, golden_luts, oracle_mod):
    """40 images of 3840x2160 in one batch: image 39's samples start at byte 39 * W * H * 16
    > 2^32. Its samples (read_samples = the batch's last image) equal the oracle's on a
    band of rows at the top, the middle and the bottom of the film."""
    from directcomputeraytracing_amd import WavefrontPathTracer
    W, H, n = 3840, 2160, 40
    assert (n - 1) * W * H * 16 > (1 << 32)
    t = WavefrontPathTracer(path_pool_size=1 << 24, iterations_per_render=16, debug_rng=True)
    try:
        s = cornell(W, H, 1)
        t.set_luts(golden_luts)
        t.on_scene_loaded(s)
        t.set_image_batch(n)
        t.clear_film()
        t.render_images(0, n)
        pos, val = t.read_samples()
        rng = t.read_rng()
        assert t.counters()["images_completed"] == n
    finally:
        t.destroy()
    flat = oracle_mod.flat_with_own_bvh(s)
    fr = oracle_mod.frame_params(s, n - 1)
    for y0 in (0, H // 2, H - 3):
        p_ref, v_ref, r_ref, _ = oracle_mod.render(flat, golden_luts, fr, oracle_mod.WAVEFRONT, rect=(0, y0, W, 3), rng=True)
        rows = slice(y0, y0 + 3)
        assert np.array_equal(rng[rows], r_ref[rows]), f"rows {y0}.."
        assert same_bits(pos[rows], p_ref[rows]).all() and same_bits(val[rows], v_ref[rows]).all(), f"rows {y0}.."


def test_upload_refuses_short_traversal_stack(native_lib, golden_luts):
    from directcomputeraytracing_amd import DCRTError, WavefrontPathTracer, _abi
    import ctypes as C
    s = cornell(32, 32, 2)
    f = s.flat()
    assert f.bvh_traversal_stack_size > 1
    g = _abi.FlatScene()
    C.pointer(g)[0] = f
    g.bvh_traversal_stack_size = f.bvh_traversal_stack_size - 1
    lib = _abi.load_library()
    t = WavefrontPathTracer(path_pool_size=1 << 12)
    try:
        rc = lib.dcrt_tracer_upload_scene(t._h, C.byref(g))
        assert rc == -1 and b"below the uploaded BVH" in lib.dcrt_last_error()
        assert lib.dcrt_tracer_upload_scene(t._h, C.byref(f)) == 0     # the exact requirement is accepted
    finally:
        t.destroy()


def test_upload_refuses_shared_child_dag(native_lib, golden_luts):
    """A node array in which interior nodes share their children (a DAG with 2^40 root-to-leaf
    paths) is refused at once as malformed (RequiredTraversalStack keeps a visited set: without
    it the walk was exponential)."""
    import ctypes as C
    import time
    from directcomputeraytracing_amd import WavefrontPathTracer, _abi
    s = cornell(16, 16, 2)
    f = s.flat()
    n = 41
    nodes = np.zeros((n, 8), np.uint32)
    box = np.array([-10, -10, -10, 10, 10, 10], np.float32).view(np.uint32)
    for i in range(n):
        nodes[i, :6] = box
        if i + 1 < n:
            nodes[i, 6] = i + 1            # right child = left child = node + 1
            nodes[i, 7] = 0                # interior, split axis 0
        else:
            nodes[i, 6] = 0                # a BLAS leaf: triangle 0, one primitive
            nodes[i, 7] = 1 << 3
    g = _abi.FlatScene()
    C.pointer(g)[0] = f
    g.bvh_nodes = nodes.ctypes.data_as(C.POINTER(_abi.BVHNode))
    g.bvh_node_count = n
    g.tlas_node_count = 0
    g.bvh_traversal_stack_size = 64
    lib = _abi.load_library()
    t = WavefrontPathTracer(path_pool_size=1 << 12)
    try:
        t0 = time.perf_counter()
        rc = lib.dcrt_tracer_upload_scene(t._h, C.byref(g))
        assert rc == -1 and b"malformed" in lib.dcrt_last_error()
        assert time.perf_counter() - t0 < 5.0
    finally:
        t.destroy()
