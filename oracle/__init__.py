"""TEST INFRASTRUCTURE ONLY -- ctypes binding of the CPU oracle (``libdcrt_oracle.so``).

The oracle is a plain-C restatement of the reference's WavefrontPathTracing.hlsl
path (see dcrt_oracle.c for per-function reference file:line citations). Only
``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg
may import this module; the product (``directcomputeraytracing_amd``) never does.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

import numpy as np

ORACLE_DIR = Path(__file__).resolve().parent
ORACLE_LIB = ORACLE_DIR / "build" / "libdcrt_oracle.so"

WAVEFRONT, MEGAKERNEL = 0, 1


class OracleCounters(C.Structure):
    _fields_ = [("extension_rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("node_visits", C.c_uint64),
                ("triangle_tests", C.c_uint64), ("blas_entries", C.c_uint64), ("shadow_node_visits", C.c_uint64),
                ("shadow_triangle_tests", C.c_uint64), ("shadow_blas_entries", C.c_uint64)]

    def as_dict(self):
        return {k: getattr(self, k) for k, _ in self._fields_}


_lib = None


def load():
    global _lib
    if _lib is not None:
        return _lib
    if not ORACLE_LIB.exists():
        import sys
        sys.path.insert(0, str(ORACLE_DIR.parent))
        from directcomputeraytracing_amd.build import build_oracle
        build_oracle()
    from directcomputeraytracing_amd import _abi as A
    lib = C.CDLL(str(ORACLE_LIB))
    P = C.POINTER
    U = C.c_uint32
    lib.oracle_render.restype = C.c_int
    lib.oracle_render.argtypes = [P(A.FlatScene), P(A.BxDFLuts), P(A.FrameParams), C.c_int, U, U, U, U,
                                  P(C.c_float), P(C.c_float), P(U), P(OracleCounters), C.c_int]
    lib.oracle_sample_convolution.restype = None
    lib.oracle_sample_convolution.argtypes = [P(A.FilterParams), U, U, P(C.c_float), P(C.c_float), P(C.c_float), U, U]
    lib.oracle_trace_rays.restype = None
    lib.oracle_trace_rays.argtypes = [P(A.FlatScene), P(A.Ray), U, P(A.RayHit), U, P(OracleCounters)]
    lib.oracle_occluded.restype = None
    lib.oracle_occluded.argtypes = [P(A.FlatScene), P(A.Ray), U, P(U), U, P(OracleCounters)]
    lib.oracle_lut_integrate.restype = None
    lib.oracle_lut_integrate.argtypes = [C.c_int, U, U, P(C.c_float)]
    lib.oracle_lut_finalize.restype = None
    lib.oracle_lut_finalize.argtypes = [P(C.c_float), P(C.c_float), P(C.c_float), P(A.BxDFLuts)]
    lib.oracle_build_luts.restype = C.c_int
    lib.oracle_build_luts.argtypes = [P(A.BxDFLuts), C.c_int]
    lib.oracle_rng_init.restype = None
    lib.oracle_rng_init.argtypes = [U, U, U, P(U)]
    lib.oracle_rng_next.restype = U
    lib.oracle_rng_next.argtypes = [P(U)]
    lib.oracle_splitmix64_pair.restype = None
    lib.oracle_splitmix64_pair.argtypes = [U, U, P(U)]
    lib.oracle_morton.restype = U
    lib.oracle_morton.argtypes = [U, U]
    lib.oracle_xoshiro_jump.restype = None
    lib.oracle_xoshiro_jump.argtypes = [P(U)]
    lib.oracle_offset_ray_origin.restype = None
    lib.oracle_offset_ray_origin.argtypes = [P(C.c_float)] * 4
    lib.oracle_generate_camera_ray.restype = None
    lib.oracle_generate_camera_ray.argtypes = [P(A.FrameParams), U, U, P(C.c_float), P(C.c_float), P(U)]
    lib.oracle_sum_log_luminance.restype = C.c_float
    lib.oracle_sum_log_luminance.argtypes = [P(C.c_float), U, U]
    lib.oracle_resolve_image.restype = None
    lib.oracle_resolve_image.argtypes = [P(C.c_float), U, U, C.c_int, C.c_int, C.c_float, C.c_float, P(C.c_float),
                                         P(C.c_uint8)]
    lib.oracle_math_eval.restype = None
    lib.oracle_math_eval.argtypes = [C.c_int, P(C.c_float), U, P(C.c_float)]
    lib.oracle_bvh_build_blas.restype = C.c_int
    lib.oracle_bvh_build_blas.argtypes = [P(A.Vertex), P(U), U, P(OracleBVHNode), P(U), P(U), P(U), P(U), P(U)]
    lib.oracle_bvh_build_tlas.restype = C.c_int
    lib.oracle_bvh_build_tlas.argtypes = [P(C.c_float), P(C.c_float), U, P(OracleBVHNode), P(U), P(U), P(U), P(U), P(U)]
    lib.oracle_bvh_pack.restype = None
    lib.oracle_bvh_pack.argtypes = [P(OracleBVHNode), U, C.c_int, P(A.BVHNode), U, U]
    lib.oracle_frame_params.restype = None
    lib.oracle_frame_params.argtypes = [P(A.SceneSettings), U, P(A.FrameParams)]
    lib.oracle_punctual_direction.restype = None
    lib.oracle_punctual_direction.argtypes = [P(C.c_float), P(C.c_float)]
    lib.oracle_bsdf_eval.restype = None
    lib.oracle_bsdf_eval.argtypes = [P(A.BxDFLuts), P(OracleBsdfMaterial), P(C.c_float), P(C.c_float), U, P(C.c_float),
                                     P(C.c_float)]
    lib.oracle_bsdf_sample.restype = None
    lib.oracle_bsdf_sample.argtypes = [P(A.BxDFLuts), P(OracleBsdfMaterial), P(C.c_float), P(C.c_float), U, P(C.c_float),
                                       P(C.c_float), P(C.c_float), P(C.c_int)]
    _lib = lib
    return lib


class OracleBsdfMaterial(C.Structure):
    _fields_ = [("type", C.c_uint32), ("albedo", C.c_float * 3), ("alpha", C.c_float), ("ior", C.c_float),
                ("two_sided", C.c_int), ("multiscattering", C.c_int), ("internal_scattering", C.c_uint32)]


def bsdf_material(type, albedo=(1.0, 1.0, 1.0), alpha=0.5, ior=1.5, two_sided=False, multiscattering=False,
                  internal_scattering=0):
    return OracleBsdfMaterial(int(type), (C.c_float * 3)(*albedo), float(alpha), float(ior), int(two_sided),
                              int(multiscattering), int(internal_scattering))


def bsdf_eval(luts, material, wi, wo):
    """EvaluateBSDF / EvaluateBSDFPdf (BSDFs.inc.hlsl:42-287) of one material in the frame
    n = (0,0,1), t = (1,0,0): (N, 3) f and (N,) pdf for (N, 3) direction pairs."""
    wi = np.ascontiguousarray(wi, np.float32).reshape(-1, 3)
    wo = np.ascontiguousarray(wo, np.float32).reshape(-1, 3)
    f = np.zeros_like(wi)
    pdf = np.zeros(len(wi), np.float32)
    load().oracle_bsdf_eval(C.byref(luts), C.byref(material), _fp(wi), _fp(wo), len(wi), _fp(f), _fp(pdf))
    return f, pdf


def bsdf_sample(luts, material, wo, u):
    """SampleBSDF (BSDFs.inc.hlsl:289-505): for (N, 3) wo and (N, 3) numbers (sx, sy, sel),
    the sampled wi (N, 3), f (N, 3), pdf (N,) and delta flags (N,)."""
    wo = np.ascontiguousarray(wo, np.float32).reshape(-1, 3)
    u = np.ascontiguousarray(u, np.float32).reshape(-1, 3)
    wi = np.zeros_like(wo)
    f = np.zeros_like(wo)
    pdf = np.zeros(len(wo), np.float32)
    delta = np.zeros(len(wo), np.int32)
    load().oracle_bsdf_sample(C.byref(luts), C.byref(material), _fp(wo), _fp(u), len(wo), _fp(wi), _fp(f), _fp(pdf),
                              delta.ctypes.data_as(C.POINTER(C.c_int)))
    return wi, f, pdf, delta.astype(bool)


class OracleBVHNode(C.Structure):
    _fields_ = [("center", C.c_float * 3), ("extents", C.c_float * 3), ("child_or_prim", C.c_uint32),
                ("count_or_instance", C.c_uint32), ("is_leaf", C.c_uint32), ("split_axis", C.c_uint32)]


_NODE_DTYPE = np.dtype([("center", np.float32, 3), ("extents", np.float32, 3), ("child_or_prim", np.uint32),
                        ("count_or_instance", np.uint32), ("is_leaf", np.uint32), ("split_axis", np.uint32)])


def build_blas(vertices, indices):
    """BVHAccel::BuildBLAS (BVHAccel.cpp:376-394), independent C restatement:
    vertices (N, 11) f32 dcrt_vertex rows, indices (T, 3). Returns the unpacked nodes
    (structured array), BVH-ordered index triples, tri_order[new] = old, depth, stack."""
    lib = load()
    from directcomputeraytracing_amd import _abi as A
    v = np.ascontiguousarray(vertices, np.float32)
    idx = np.ascontiguousarray(indices, np.uint32).reshape(-1)
    n = idx.size // 3
    nodes = np.zeros(max(1, 2 * n), _NODE_DTYPE)
    out_idx = np.zeros(idx.size, np.uint32)
    order = np.zeros(n, np.uint32)
    cnt, depth, stack = C.c_uint32(), C.c_uint32(), C.c_uint32()
    rc = lib.oracle_bvh_build_blas(v.ctypes.data_as(C.POINTER(A.Vertex)), _up(idx), n,
                                   nodes.ctypes.data_as(C.POINTER(OracleBVHNode)), C.byref(cnt), _up(out_idx),
                                   _up(order), C.byref(depth), C.byref(stack))
    if rc != 0:
        raise ValueError("oracle_bvh_build_blas: empty mesh")
    return {"nodes": nodes[:cnt.value].copy(), "indices": out_idx.reshape(-1, 3), "order": order,
            "max_depth": depth.value, "max_stack_size": stack.value}


def pack_bvh(nodes, is_blas, node_offset=0, prim_offset=0):
    """BVHAccel::PackBVH (BVHAccel.cpp:413-447) -> (N, 8) uint32 (the 32-B GPU node)."""
    lib = load()
    from directcomputeraytracing_amd import _abi as A
    nodes = np.ascontiguousarray(nodes, _NODE_DTYPE)
    out = np.zeros((len(nodes), 8), np.uint32)
    lib.oracle_bvh_pack(nodes.ctypes.data_as(C.POINTER(OracleBVHNode)), len(nodes), int(is_blas),
                        out.ctypes.data_as(C.POINTER(A.BVHNode)), node_offset, prim_offset)
    return out


def build_scene_bvh(meshes, instances):
    """The BVH half of CScene::LoadFromFile (Scene.cpp:160-215, 337-421, 431-434): BLAS
    per mesh, TLAS over the instances' transformed BLAS-root boxes, the TLAS leaves
    patched to their BLAS roots and instance numbers, everything packed.

    meshes: [{"vertices" (N, 11), "indices" (T, 3) load order, "material_ids" (T,)}];
    instances: [(mesh_index, transform (4, 3) XMFLOAT4X3)] in load order.
    Returns nodes (N, 8) u32, triangles (T, 3) u32 (global vertex indices),
    material_ids, instance_order (reordered -> original), stack_size and the forward
    instance transforms (I, 12) as Scene.cpp:429-434 stores them."""
    lib = load()
    blas = [build_blas(m["vertices"], m["indices"]) for m in meshes]
    ni = len(instances)
    boxes = np.zeros((ni, 6), np.float32)
    xf = np.zeros((ni, 12), np.float32)
    for i, (mesh, t) in enumerate(instances):
        root = blas[mesh]["nodes"][0]
        boxes[i, :3], boxes[i, 3:] = root["center"], root["extents"]
        xf[i] = np.asarray(t, np.float32).reshape(12)
    tnodes = np.zeros(max(1, 2 * ni), _NODE_DTYPE)
    order = np.zeros(ni, np.uint32)
    depths = np.zeros(ni, np.uint32)
    cnt, depth, stack = C.c_uint32(), C.c_uint32(), C.c_uint32()
    if lib.oracle_bvh_build_tlas(_fp(boxes), _fp(xf), ni, tnodes.ctypes.data_as(C.POINTER(OracleBVHNode)), C.byref(cnt),
                                 _up(order), C.byref(depth), C.byref(stack), _up(depths)) != 0:
        raise ValueError("oracle_bvh_build_tlas: no instances")
    tlas = tnodes[:cnt.value].copy()
    stack_size = max(int(depths[r]) + blas[instances[int(order[r])][0]]["max_depth"] for r in range(ni))
    parts, blas_offsets = [], []
    node_offset, tri_offset = len(tlas), 0
    for m, b in zip(meshes, blas):
        parts.append(pack_bvh(b["nodes"], True, node_offset, tri_offset))
        blas_offsets.append(node_offset)
        node_offset += len(b["nodes"])
        tri_offset += len(m["indices"])
    for node in tlas:
        if node["count_or_instance"] > 0:   # a leaf: its instance's BLAS root and number
            prim = int(node["child_or_prim"])
            node["child_or_prim"] = blas_offsets[instances[int(order[prim])][0]]
            node["count_or_instance"] = prim
    nodes = np.concatenate([pack_bvh(tlas, False)] + parts)
    tris, mats, voff = [], [], 0
    for m, b in zip(meshes, blas):
        tris.append(b["indices"].astype(np.uint32) + np.uint32(voff))
        mats.append(np.asarray(m["material_ids"], np.uint32)[b["order"]])
        voff += len(m["vertices"])
    fwd = np.zeros((ni, 12), np.float32)
    for r in range(ni):
        t = xf[int(order[r])].reshape(4, 3)
        fwd[r] = t.T.reshape(12)     # XMFLOAT4X3(_11, _21, _31, _41, _12, ...)
    return {"nodes": nodes, "triangles": np.concatenate(tris) if tris else np.zeros((0, 3), np.uint32),
            "material_ids": np.concatenate(mats) if mats else np.zeros(0, np.uint32), "instance_order": order,
            "stack_size": stack_size, "forward_transforms": fwd, "tlas_node_count": len(tlas)}


def _fp(a):
    return a.ctypes.data_as(C.POINTER(C.c_float))


def _up(a):
    return a.ctypes.data_as(C.POINTER(C.c_uint32))


def default_threads() -> int:
    return max(1, min(int(os.environ.get("OMP_NUM_THREADS", "0") or 0) or (os.cpu_count() or 1), 16))


def render(flat, luts, frame, mode=WAVEFRONT, rect=None, rng=False, threads=None):
    """Render one image (frame.frame_seed) over `rect` (x0, y0, w, h); returns
    (sample_position HxWx2, sample_value HxWx4, rng HxWx4 or None, counters)."""
    lib = load()
    W, H = frame.resolution[0], frame.resolution[1]
    x0, y0, w, h = rect or (0, 0, W, H)
    pos = np.zeros((H, W, 2), np.float32)
    val = np.zeros((H, W, 4), np.float32)
    st = np.zeros((H, W, 4), np.uint32) if rng else None
    cnt = OracleCounters()
    rc = lib.oracle_render(C.byref(flat), C.byref(luts), C.byref(frame), mode, x0, y0, w, h, _fp(pos), _fp(val),
                           _up(st) if st is not None else None, C.byref(cnt), threads or default_threads())
    if rc != 0:
        raise RuntimeError(f"oracle_render failed: {rc}")
    return pos, val, st, cnt.as_dict()


def sample_convolution(filter_params, pos, val, film=None, rows=None):
    lib = load()
    H, W = pos.shape[:2]
    film = np.zeros((H, W, 4), np.float32) if film is None else film
    r0, r1 = rows or (0, H)
    lib.oracle_sample_convolution(C.byref(filter_params), W, H, _fp(np.ascontiguousarray(pos)),
                                  _fp(np.ascontiguousarray(val)), _fp(film), r0, r1)
    return film


def trace_rays(flat, rays, features):
    from directcomputeraytracing_amd import _abi as A
    from directcomputeraytracing_amd.tracer import HIT_DTYPE
    lib = load()
    hits = np.zeros(len(rays), HIT_DTYPE)
    cnt = OracleCounters()
    lib.oracle_trace_rays(C.byref(flat), rays.ctypes.data_as(C.POINTER(A.Ray)), len(rays),
                          hits.ctypes.data_as(C.POINTER(A.RayHit)), features, C.byref(cnt))
    return hits, cnt.as_dict()


def occluded(flat, rays, features):
    from directcomputeraytracing_amd import _abi as A
    lib = load()
    out = np.zeros(len(rays), np.uint32)
    cnt = OracleCounters()
    lib.oracle_occluded(C.byref(flat), rays.ctypes.data_as(C.POINTER(A.Ray)), len(rays), _up(out), features,
                        C.byref(cnt))
    return out, cnt.as_dict()


def build_luts(threads=None):
    from directcomputeraytracing_amd import _abi as A
    lib = load()
    luts = A.BxDFLuts()
    if lib.oracle_build_luts(C.byref(luts), threads or default_threads()) != 0:
        raise RuntimeError("oracle_build_luts failed")
    return luts


def luts_to_arrays(luts) -> dict:
    return {name: np.ctypeslib.as_array(getattr(luts, name)).copy() for name, _ in luts._fields_}


def luts_from_arrays(arrays: dict):
    from directcomputeraytracing_amd import _abi as A
    luts = A.BxDFLuts()
    for name, _ in luts._fields_:
        dst = np.ctypeslib.as_array(getattr(luts, name))
        dst[:] = np.asarray(arrays[name], np.uint16).reshape(dst.shape)
    return luts


def rng_init(px, py, seed):
    lib = load()
    s = np.zeros(4, np.uint32)
    lib.oracle_rng_init(px, py, seed, _up(s))
    return s


def rng_next(state):
    return load().oracle_rng_next(_up(state))


def splitmix64_pair(lo, hi):
    out = np.zeros(6, np.uint32)
    load().oracle_splitmix64_pair(lo, hi, _up(out))
    return out


def morton(x, y):
    return load().oracle_morton(x, y)


def math_eval(function, x):
    x = np.ascontiguousarray(x, np.float32)
    y = np.empty_like(x)
    load().oracle_math_eval(function, _fp(x), x.size, _fp(y))
    return y


def camera_ray(frame, px, py):
    o = np.zeros(3, np.float32)
    d = np.zeros(3, np.float32)
    r = np.zeros(4, np.uint32)
    load().oracle_generate_camera_ray(C.byref(frame), px, py, _fp(o), _fp(d), _up(r))
    return o, d, r


def resolve_image(film, params, thresholds):
    """PostProcessings.hlsl + SumLuminance.hlsl restated: H x W x 4 sRGB8."""
    film = np.ascontiguousarray(film, np.float32)
    H, W = film.shape[:2]
    out = np.empty((H, W, 4), np.uint8)
    th = np.ascontiguousarray(thresholds, np.float32)
    load().oracle_resolve_image(_fp(film), W, H, params.enabled, params.auto_exposure, params.ev100,
                                params.luminance_white, _fp(th), out.ctypes.data_as(C.POINTER(C.c_uint8)))
    return out


def sum_log_luminance(film):
    film = np.ascontiguousarray(film, np.float32)
    return load().oracle_sum_log_luminance(_fp(film), film.shape[1], film.shape[0])


# ---- the oracle's own CScene flattening (Scene.cpp:423-552, 672-807; WavefrontPathTracer.cpp:372-428) ----
# Driven from the scene state the loaders produced (dcrt_scene_get_settings / _material_setting /
# _mesh_light / _punctual_light / _instance_material_override, dcrt_scene_get_loaded_mesh /
# _instance): everything the reference's flattening derives from it is restated here, separately
# from csrc/host/scene.cpp. The texture texels and the environment cube are loader outputs and are
# taken as loaded.

def f32_from_fraction(x) -> np.float32:
    """An exact rational rounded to the nearest float32 (ties to even), as one IEEE operation
    would round it (no double rounding through float64)."""
    import math
    from fractions import Fraction
    x = Fraction(x)
    if x == 0:
        return np.float32(0.0)
    neg = x < 0
    n, d = abs(x.numerator), x.denominator
    e = n.bit_length() - d.bit_length()          # 2^e <= |x| < 2^(e+1) after the correction
    if (n << max(0, -e)) < (d << max(0, e)):
        e -= 1
    e = max(e, -126)                              # subnormals share the minimum exponent
    shift = 23 - e                                # |x| * 2^shift: the 24-bit significand
    num, den = (n << shift, d) if shift >= 0 else (n, d << -shift)
    m, r = divmod(num, den)
    if 2 * r > den or (2 * r == den and m & 1):
        m += 1
    v = math.ldexp(m, e - 23)
    if v >= 2.0 ** 128:
        v = math.inf
    return np.float32(-v if neg else v)


def inverse_affine_exact(t43) -> np.ndarray:
    """XMMatrixInverse of an XMFLOAT4X3 instance transform (row vectors: rows 0-2 the linear
    part A, row 3 the translation t), as the exactly rounded inverse [[A^-1, 0], [-t A^-1, 1]]:
    (4, 3) float32. DirectXMath's own float arithmetic is not available here: parity unpinned;
    this is the exactly rounded value of what it approximates."""
    from fractions import Fraction
    M = [[Fraction(float(v)) for v in row] for row in np.asarray(t43, np.float32).reshape(4, 3)]
    a = M[:3]
    det = (a[0][0] * (a[1][1] * a[2][2] - a[1][2] * a[2][1]) - a[0][1] * (a[1][0] * a[2][2] - a[1][2] * a[2][0])
           + a[0][2] * (a[1][0] * a[2][1] - a[1][1] * a[2][0]))
    out = np.zeros((4, 3), np.float32)
    if det == 0:
        return out
    inv = [[None] * 3 for _ in range(3)]
    for r in range(3):
        for c in range(3):
            rows = [i for i in range(3) if i != c]
            cols = [j for j in range(3) if j != r]
            minor = a[rows[0]][cols[0]] * a[rows[1]][cols[1]] - a[rows[0]][cols[1]] * a[rows[1]][cols[0]]
            inv[r][c] = (minor if (r + c) % 2 == 0 else -minor) / det
    t = M[3]
    for r in range(3):
        for c in range(3):
            out[r, c] = f32_from_fraction(inv[r][c])
    for c in range(3):
        out[3, c] = f32_from_fraction(-(t[0] * inv[0][c] + t[1] * inv[1][c] + t[2] * inv[2][c]))
    return out


def _clamp01(v) -> np.float32:   # std::clamp(v, 0.f, 1.f): NaN passes through
    v = np.float32(v)
    return np.float32(0.0) if v < 0 else (np.float32(1.0) if v > 1 else v)


def frame_params(scene, frame_seed: int = 0):
    """The frame constants Render() uploads (WavefrontPathTracer.cpp:372-428), from the scene
    state: camera matrix, film distance, aperture, blade vertex, light count (C restatement,
    dcrt_oracle_scene.c)."""
    from directcomputeraytracing_amd import _abi as A
    out = A.FrameParams()
    settings = scene.settings()
    load().oracle_frame_params(C.byref(settings), int(frame_seed), C.byref(out))
    return out


def flatten_scene(scene):
    """The flattened scene (dcrt_flat_scene: Scene.cpp:273-608 uploads plus UpdateLight /
    Material / InstanceFlagsGPUData, Scene.cpp:672-807), built by the oracle from the scene
    state alone: its own BVHAccel build (build_scene_bvh), its own light array, material
    translation, instance arrays and inverse transforms. The returned FlatScene keeps its
    arrays alive."""
    from directcomputeraytracing_amd import _abi as A
    lib = load()
    meshes, instances = scene.loaded_content()
    own = build_scene_bvh(meshes, instances)
    settings = scene.settings()
    order = [int(i) for i in own["instance_order"]]               # reordered -> original
    reordered = {orig: r for r, orig in enumerate(order)}          # original -> reordered
    overrides = scene.instance_material_overrides()
    mats = [scene.material_setting(i) for i in range(settings.material_count)]

    # materials (UpdateMaterialGPUData, Scene.cpp:742-774): a conductor's albedo slot carries k
    materials = np.zeros((len(mats), 13), np.uint32)
    mf = materials.view(np.float32)
    for i, m in enumerate(mats):
        albedo = m.k if m.material_type == A.MATERIAL_CONDUCTOR else m.albedo
        mf[i, 0:3] = np.array(albedo[:], np.float32)
        tex = -1 if m.material_type in (A.MATERIAL_CONDUCTOR, A.MATERIAL_DIELECTRIC) else m.albedo_texture_index
        materials[i, 3] = np.uint32(tex & 0xFFFFFFFF)
        mf[i, 4:7] = np.array(m.ior[:], np.float32)
        mf[i, 7] = _clamp01(m.roughness)
        mf[i, 8:10] = np.array(m.tiling[:], np.float32)
        mf[i, 10] = np.float32(m.opacity)
        flags = m.material_type & 0xF
        flags |= 0x80 if m.multiscattering else 0
        flags |= 0x40 if m.is_two_sided else 0
        flags |= 0x20 if m.has_roughness_texture else 0
        flags |= (m.internal_scattering_mode << 8) & 0x300
        materials[i, 11] = flags
        materials[i, 12] = np.uint32(m.opacity_texture_index & 0xFFFFFFFF)

    def is_opaque(i):   # SMaterial::IsOpaque (Scene.cpp:57-60)
        return np.float32(mats[i].opacity) == np.float32(1.0) and mats[i].opacity_texture_index == -1

    # mesh flags (Scene.cpp:62-90): opaque when every triangle's material is
    mesh_opaque = [all(is_opaque(int(i)) for i in m["material_ids"]) for m in meshes]
    ni = len(instances)
    # instance arrays in TLAS (reordered) order (Scene.cpp:423-552, 776-807)
    transforms = np.zeros((2 * ni, 12), np.float32)
    flags = np.zeros(ni, np.uint32)
    ovr = np.zeros(ni, np.uint32)
    for r, orig in enumerate(order):
        mesh, t = instances[orig]
        t = np.asarray(t, np.float32).reshape(4, 3)
        inv = inverse_affine_exact(t)
        transforms[r] = t.T.reshape(12)          # XMFLOAT4X3(_11, _21, _31, _41, _12, ...)
        transforms[ni + r] = inv.T.reshape(12)
        o = overrides[orig]
        opaque = is_opaque(o) if o != 0xFFFFFFFF else mesh_opaque[mesh]
        flags[r] = 1 if opaque else 0
        ovr[r] = o
    # mesh lights, then the environment light, then the punctual lights (Scene.cpp:672-735);
    # each instance's light index (Scene.cpp:467-499)
    mesh_lights = scene.mesh_lights()
    tri_offsets = np.concatenate([[0], np.cumsum([len(m["indices"]) for m in meshes])]).astype(np.uint32)
    lights = []
    light_index = np.full(ni, 0xFFFFFFFF, np.uint32)
    for li, (inst, color) in enumerate(mesh_lights):
        mesh = instances[inst][0]
        rec = np.zeros(7, np.uint32)
        rec[0:3] = np.array(color, np.float32).view(np.uint32)
        rec[3] = tri_offsets[mesh]
        rec[4] = len(meshes[mesh]["indices"])
        rec[5] = reordered[inst]
        rec[6] = 0x2
        lights.append(rec)
        light_index[reordered[inst]] = li
    if settings.has_environment_light:
        rec = np.zeros(7, np.uint32)
        rec[0:3] = np.array(settings.environment_color[:], np.float32).view(np.uint32)
        rec[6] = 0x8
        lights.append(rec)
    for pos, euler, color, directional in scene.punctual_lights():
        rec = np.zeros(7, np.uint32)
        rec[0:3] = np.array(color, np.float32).view(np.uint32)
        if directional:
            e = (C.c_float * 3)(*euler)
            d = (C.c_float * 3)()
            lib.oracle_punctual_direction(e, d)
            rec[3:6] = np.array(d[:], np.float32).view(np.uint32)
        else:
            rec[3:6] = np.array(pos, np.float32).view(np.uint32)
        rec[6] = 0x4 if directional else 0x1
        lights.append(rec)
    lights = np.array(lights, np.uint32).reshape(-1, 7)
    vertices = np.ascontiguousarray(np.concatenate([m["vertices"] for m in meshes]), np.float32)
    keep = {"vertices": vertices, "nodes": np.ascontiguousarray(own["nodes"], np.uint32),
            "triangles": np.ascontiguousarray(own["triangles"], np.uint32),
            "material_ids": np.ascontiguousarray(own["material_ids"], np.uint32),
            "transforms": transforms, "light_index": light_index, "flags": flags, "overrides": ovr,
            "materials": materials, "lights": lights if len(lights) else np.zeros((1, 7), np.uint32)}
    src = scene.flat()   # only for the loaders' texture texels
    f = A.FlatScene()
    f.vertices = keep["vertices"].ctypes.data_as(C.POINTER(A.Vertex))
    f.vertex_count = vertices.shape[0]
    f.triangles = keep["triangles"].ctypes.data_as(C.POINTER(C.c_uint32))
    f.triangle_count = keep["triangles"].shape[0]
    f.bvh_nodes = keep["nodes"].ctypes.data_as(C.POINTER(A.BVHNode))
    f.bvh_node_count = keep["nodes"].shape[0]
    f.tlas_node_count = own["tlas_node_count"]
    f.material_ids = keep["material_ids"].ctypes.data_as(C.POINTER(C.c_uint32))
    f.instance_transforms = keep["transforms"].ctypes.data_as(C.POINTER(A.Float4x3))
    f.instance_count = ni
    f.instance_light_indices = keep["light_index"].ctypes.data_as(C.POINTER(C.c_uint32))
    f.instance_flags = keep["flags"].ctypes.data_as(C.POINTER(C.c_uint32))
    f.instance_material_overrides = keep["overrides"].ctypes.data_as(C.POINTER(C.c_uint32))
    f.materials = keep["materials"].ctypes.data_as(C.POINTER(A.Material))
    f.material_count = len(mats)
    f.lights = keep["lights"].ctypes.data_as(C.POINTER(A.Light))
    f.light_count = len(lights)
    f.environment_light_index = len(mesh_lights) if settings.has_environment_light else 0xFFFFFFFF
    f.textures = src.textures
    f.texture_count = src.texture_count
    f.env_cube_rgb = settings.env_cube_rgb if settings.env_cube_size else None
    f.env_cube_size = settings.env_cube_size
    f.bvh_traversal_stack_size = own["stack_size"]
    f._keep = (keep, scene)
    return f


def flat_with_own_bvh(scene):
    """The oracle side of every GPU parity test: the scene flattened by the oracle alone
    (flatten_scene -- its own BVHAccel build, lights, materials, instance arrays)."""
    return flatten_scene(scene)
