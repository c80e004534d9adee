"""ctypes mirror of ``include/dcrt.h`` (the C ABI of the MI355X tracer).

Only plain C types cross the boundary; numpy is used for host views of the
flattened scene buffers. Loading fails loudly when the native library is
missing: there is no CPU fallback for the product path.
"""
from __future__ import annotations

import ctypes as C
import os
from pathlib import Path

PKG_DIR = Path(__file__).resolve().parent
LIB_PATH = PKG_DIR / "libdcrt.so"

# ---- status codes / flags (dcrt.h) -----------------------------------------
DCRT_OK = 0
ABI_VERSION = 2          # DCRT_ABI_VERSION: load_library refuses a libdcrt.so of another
ERRORS = {-1: "DCRT_E_INVALID_ARG", -2: "DCRT_E_HIP", -3: "DCRT_E_NO_SCENE", -4: "DCRT_E_IO",
          -5: "DCRT_E_LIMIT", -6: "DCRT_E_NO_DEVICE"}
LIGHT_INDEX_INVALID = 0xFFFFFFFF
FEATURE_GGX_SAMPLE_VNDF = 0x01
FEATURE_NO_FRONT_TO_BACK = 0x02
FEATURE_LIGHT_VISIBLE = 0x04
FEATURE_WATERTIGHT = 0x08
FEATURE_ALLOW_ANYHIT = 0x10
FEATURE_DEFAULT = FEATURE_GGX_SAMPLE_VNDF | FEATURE_LIGHT_VISIBLE | FEATURE_WATERTIGHT
FILTER_BOX, FILTER_TRIANGLE, FILTER_GAUSSIAN, FILTER_MITCHELL, FILTER_LANCZOS = range(5)
MATERIAL_DIFFUSE, MATERIAL_PLASTIC, MATERIAL_CONDUCTOR, MATERIAL_DIELECTRIC, MATERIAL_THIN_DIELECTRIC = range(5)


class Vertex(C.Structure):
    _fields_ = [("position", C.c_float * 3), ("normal", C.c_float * 3), ("tangent", C.c_float * 3),
                ("texcoord", C.c_float * 2)]


class BVHNode(C.Structure):
    _fields_ = [("bbox_min", C.c_float * 3), ("bbox_max", C.c_float * 3), ("right_child_or_prim_index", C.c_uint32),
                ("misc", C.c_uint32)]


class Material(C.Structure):
    _fields_ = [("albedo", C.c_float * 3), ("albedo_texture_index", C.c_int32), ("ior", C.c_float * 3),
                ("roughness", C.c_float), ("tex_tiling", C.c_float * 2), ("opacity", C.c_float),
                ("flags", C.c_uint32), ("opacity_texture_index", C.c_int32)]


class Light(C.Structure):
    _fields_ = [("radiance", C.c_float * 3), ("position_or_triangle_range", C.c_float * 3), ("flags", C.c_uint32)]


class Float4x3(C.Structure):
    _fields_ = [("m", C.c_float * 12)]


class Texture(C.Structure):
    _fields_ = [("width", C.c_uint32), ("height", C.c_uint32), ("format", C.c_uint32),
                ("pixels", C.POINTER(C.c_uint8))]


class FlatScene(C.Structure):
    _fields_ = [
        ("vertices", C.POINTER(Vertex)), ("vertex_count", C.c_uint32),
        ("triangles", C.POINTER(C.c_uint32)), ("triangle_count", C.c_uint32),
        ("bvh_nodes", C.POINTER(BVHNode)), ("bvh_node_count", C.c_uint32),
        ("tlas_node_count", C.c_uint32),
        ("material_ids", C.POINTER(C.c_uint32)),
        ("instance_transforms", C.POINTER(Float4x3)), ("instance_count", C.c_uint32),
        ("instance_light_indices", C.POINTER(C.c_uint32)),
        ("instance_flags", C.POINTER(C.c_uint32)),
        ("instance_material_overrides", C.POINTER(C.c_uint32)),
        ("materials", C.POINTER(Material)), ("material_count", C.c_uint32),
        ("lights", C.POINTER(Light)), ("light_count", C.c_uint32),
        ("environment_light_index", C.c_uint32),
        ("textures", C.POINTER(Texture)), ("texture_count", C.c_uint32),
        ("env_cube_rgb", C.POINTER(C.c_float)), ("env_cube_size", C.c_uint32),
        ("bvh_traversal_stack_size", C.c_uint32),
    ]


class BxDFLuts(C.Structure):
    _fields_ = [("brdf", C.c_uint16 * (32 * 32)), ("brdf_avg", C.c_uint16 * 32),
                ("brdf_dielectric", C.c_uint16 * (32 * 16 * 32)), ("brdf_dielectric_avg", C.c_uint16 * (16 * 16 * 2)),
                ("bsdf", C.c_uint16 * (32 * 16 * 32)), ("bsdf_avg", C.c_uint16 * (16 * 16 * 2))]


class FrameParams(C.Structure):
    _fields_ = [("camera_transform", C.c_float * 16), ("resolution", C.c_uint32 * 2), ("film_size", C.c_float * 2),
                ("aperture_radius", C.c_float), ("focal_distance", C.c_float), ("film_distance", C.c_float),
                ("blade_count", C.c_uint32), ("blade_vertex_pos", C.c_float * 2), ("aperture_base_angle", C.c_float),
                ("frame_seed", C.c_uint32), ("max_bounce_count", C.c_uint32), ("light_count", C.c_uint32),
                ("environment_light_index", C.c_uint32), ("features", C.c_uint32)]


class FilterParams(C.Structure):
    _fields_ = [("filter", C.c_uint32), ("radius", C.c_float), ("gaussian_alpha", C.c_float),
                ("mitchell_b", C.c_float), ("mitchell_c", C.c_float), ("lanczos_tau", C.c_uint32)]


class Ray(C.Structure):
    _fields_ = [("origin", C.c_float * 3), ("t_max", C.c_float), ("direction", C.c_float * 3), ("t_min", C.c_float)]


class RayHit(C.Structure):
    _fields_ = [("t", C.c_float), ("u", C.c_float), ("v", C.c_float), ("triangle_id", C.c_uint32),
                ("instance_index", C.c_uint32)]


class PostFxParams(C.Structure):
    _fields_ = [("enabled", C.c_int32), ("auto_exposure", C.c_int32), ("ev100", C.c_float), ("luminance_white", C.c_float)]


class TracerConfig(C.Structure):
    _fields_ = [("path_pool_size", C.c_uint32), ("iterations_per_render", C.c_uint32), ("device", C.c_int32),
                ("stream", C.c_void_p), ("debug_rng", C.c_uint32)]


class RayStats(C.Structure):
    _fields_ = [("extension_rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("new_paths", C.c_uint64),
                ("iterations", C.c_uint64), ("images_completed", C.c_uint64)]


class FilmPartition(C.Structure):
    _fields_ = [("world_size", C.c_uint32), ("rank", C.c_uint32), ("stripe_height", C.c_uint32),
                ("halo_rows", C.c_uint32)]


class TraversalStats(C.Structure):
    _fields_ = [("ext_node_visits", C.c_uint64), ("ext_triangle_tests", C.c_uint64), ("ext_blas_entries", C.c_uint64),
                ("shadow_node_visits", C.c_uint64), ("shadow_triangle_tests", C.c_uint64),
                ("shadow_blas_entries", C.c_uint64), ("ext_launches", C.c_uint64), ("ext_kernel_ms", C.c_double),
                ("ext_max_node_visits", C.c_uint64), ("shadow_max_node_visits", C.c_uint64),
                ("material_launches", C.c_uint64), ("material_kernel_ms", C.c_double),
                ("control_launches", C.c_uint64), ("control_kernel_ms", C.c_double)]


class TracerInfo(C.Structure):
    _fields_ = [("path_pool_size", C.c_uint32), ("scene_in_lds", C.c_uint32), ("cached_nodes", C.c_uint32),
                ("cached_triangles", C.c_uint32), ("cast_block", C.c_uint32), ("traversal_stack", C.c_uint32),
                ("material_generic", C.c_uint32), ("pair_traversal", C.c_uint32), ("control_grid", C.c_uint32),
                ("material_grid", C.c_uint32), ("cast_grid", C.c_uint32), ("material_lds", C.c_uint32),
                ("cast_identity", C.c_uint32), ("stack_lds_rows", C.c_uint32), ("ring_rows", C.c_uint32),
                ("cast_waves_per_cu", C.c_uint32)]


class MaterialSetting(C.Structure):
    _fields_ = [("albedo", C.c_float * 3), ("roughness", C.c_float), ("ior", C.c_float * 3), ("opacity", C.c_float),
                ("k", C.c_float * 3), ("tiling", C.c_float * 2), ("material_type", C.c_uint32),
                ("albedo_texture_index", C.c_int32), ("opacity_texture_index", C.c_int32),
                ("internal_scattering_mode", C.c_uint32), ("multiscattering", C.c_uint32),
                ("is_two_sided", C.c_uint32), ("has_roughness_texture", C.c_uint32)]


class SceneSettings(C.Structure):
    _fields_ = [("resolution", C.c_uint32 * 2), ("max_bounce_count", C.c_uint32), ("camera_type", C.c_uint32),
                ("fov_x", C.c_float), ("focal_length", C.c_float), ("focal_distance", C.c_float),
                ("relative_aperture", C.c_float), ("aperture_blade_count", C.c_uint32), ("aperture_rotation", C.c_float),
                ("film_size", C.c_float * 2), ("camera_position", C.c_float * 3), ("camera_euler_angles", C.c_float * 3),
                ("features", C.c_uint32), ("has_environment_light", C.c_uint32), ("environment_color", C.c_float * 3),
                ("env_cube_rgb", C.POINTER(C.c_float)), ("env_cube_size", C.c_uint32),
                ("mesh_light_count", C.c_uint32), ("punctual_light_count", C.c_uint32),
                ("material_count", C.c_uint32), ("texture_count", C.c_uint32)]


class ObjMesh(C.Structure):
    _fields_ = [("vertices", C.POINTER(Vertex)), ("vertex_count", C.c_uint32), ("indices", C.POINTER(C.c_uint32)),
                ("material_ids", C.POINTER(C.c_uint32)), ("triangle_count", C.c_uint32)]


class ObjMaterial(C.Structure):
    _fields_ = [("albedo", C.c_float * 3), ("ior", C.c_float), ("roughness", C.c_float), ("opacity", C.c_float),
                ("albedo_texture_index", C.c_int32), ("opacity_texture_index", C.c_int32)]


OBJ_SCENE_LAYOUT = 1

# Every symbol include/dcrt.h declares: (name, restype, argtypes)
_P = C.c_void_p
_I = C.c_int
_U = C.c_uint32
_FP = C.POINTER(C.c_float)
SIGNATURES = [
    ("dcrt_abi_version", _I, []),
    ("dcrt_version", C.c_char_p, []),
    ("dcrt_last_error", C.c_char_p, []),
    ("dcrt_device_count", _I, [C.POINTER(C.c_int)]),
    ("dcrt_scene_create", _I, [C.POINTER(_P)]),
    ("dcrt_scene_destroy", None, [_P]),
    ("dcrt_scene_reset", _I, [_P, _U, _U]),
    ("dcrt_scene_load_from_file", _I, [_P, C.c_char_p]),
    ("dcrt_scene_add_punctual_light", _I, [_P, _FP, _FP, _FP, _I]),
    ("dcrt_scene_set_environment_light", _I, [_P, _FP, _FP, _U]),
    ("dcrt_scene_set_camera", _I, [_P, _FP, _FP]),
    ("dcrt_scene_set_lens", _I, [_P, _I, C.c_float, C.c_float, C.c_float, C.c_float, _U, C.c_float, _FP]),
    ("dcrt_scene_set_max_bounce", _I, [_P, _U]),
    ("dcrt_scene_set_filter", _I, [_P, C.POINTER(FilterParams)]),
    ("dcrt_scene_get_filter", _I, [_P, C.POINTER(FilterParams)]),
    ("dcrt_scene_get_resolution", _I, [_P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    ("dcrt_scene_get_material_count", _I, [_P, C.POINTER(C.c_uint32)]),
    ("dcrt_scene_set_material", _I, [_P, _U, _I, _FP, C.c_float, _FP, _FP, _I, _I]),
    ("dcrt_scene_set_material_opacity", _I, [_P, _U, C.c_float, C.c_int32]),
    ("dcrt_scene_get_material_setting", _I, [_P, _U, C.POINTER(MaterialSetting)]),
    ("dcrt_scene_set_material_multiscattering", _I, [_P, _U, _I]),
    ("dcrt_scene_get_settings", _I, [_P, C.POINTER(SceneSettings)]),
    ("dcrt_scene_get_mesh_light", _I, [_P, _U, C.POINTER(C.c_uint32), _FP]),
    ("dcrt_scene_get_punctual_light", _I, [_P, _U, _FP, _FP, _FP, C.POINTER(C.c_int)]),
    ("dcrt_scene_get_instance_material_override", _I, [_P, _U, C.POINTER(C.c_uint32)]),
    ("dcrt_scene_set_features", _I, [_P, _U]),
    ("dcrt_scene_get_features", _I, [_P, C.POINTER(C.c_uint32)]),
    ("dcrt_scene_get_flat", _I, [_P, C.POINTER(FlatScene)]),
    ("dcrt_scene_get_frame_params", _I, [_P, _U, C.POINTER(FrameParams)]),
    ("dcrt_scene_get_bvh_info", _I, [_P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    ("dcrt_bvh_build_blas", _I, [C.POINTER(Vertex), C.POINTER(C.c_uint32), _U, C.POINTER(BVHNode),
                                 C.POINTER(C.c_uint32), C.POINTER(C.c_uint32), C.POINTER(C.c_uint32),
                                 C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    ("dcrt_scene_get_content_counts", _I, [_P, C.POINTER(C.c_uint32), C.POINTER(C.c_uint32)]),
    ("dcrt_scene_get_loaded_mesh", _I, [_P, _U, C.POINTER(ObjMesh)]),
    ("dcrt_scene_get_instance", _I, [_P, _U, C.POINTER(C.c_uint32), _FP]),
    ("dcrt_obj_load", _I, [C.c_char_p, _U, _U, C.POINTER(_P)]),
    ("dcrt_obj_mesh_count", _I, [_P, C.POINTER(C.c_uint32)]),
    ("dcrt_obj_get_mesh", _I, [_P, _U, C.POINTER(ObjMesh)]),
    ("dcrt_obj_material_count", _I, [_P, C.POINTER(C.c_uint32)]),
    ("dcrt_obj_get_material", _I, [_P, _U, C.POINTER(ObjMaterial)]),
    ("dcrt_obj_free", None, [_P]),
    ("dcrt_xml_dump_tree", _I, [C.c_char_p, C.c_char_p, _U, C.POINTER(C.c_uint32)]),
    ("dcrt_tracer_create", _I, [C.POINTER(TracerConfig), C.POINTER(_P)]),
    ("dcrt_tracer_destroy", None, [_P]),
    ("dcrt_tracer_upload_scene", _I, [_P, C.POINTER(FlatScene)]),
    ("dcrt_tracer_set_frame_params", _I, [_P, C.POINTER(FrameParams)]),
    ("dcrt_tracer_set_film_partition", _I, [_P, C.POINTER(FilmPartition)]),
    ("dcrt_tracer_set_film_bands", _I, [_P, C.POINTER(C.c_uint32), _U, _U]),
    ("dcrt_tracer_set_row_cost_probe", _I, [_P, _I]),
    ("dcrt_tracer_read_row_cost", _I, [_P, C.POINTER(C.c_uint32)]),
    ("dcrt_tracer_render", _I, [_P, _U]),
    ("dcrt_tracer_render_images", _I, [_P, _U, _U, C.POINTER(FilterParams)]),
    ("dcrt_tracer_render_images_strided", _I, [_P, _U, _U, _U, _I, C.POINTER(FilterParams)]),
    ("dcrt_tracer_image_sample_ptrs", _I, [_P, _U, C.POINTER(_P), C.POINTER(_P)]),
    ("dcrt_tracer_accumulate_images", _I, [_P, C.POINTER(_P), C.POINTER(_P), _U, C.POINTER(FilterParams)]),
    ("dcrt_tracer_set_mode", _I, [_P, _I]),
    ("dcrt_tracer_set_image_batch", _I, [_P, C.c_uint32]),
    ("dcrt_tracer_reset_image", _I, [_P]),
    ("dcrt_tracer_is_image_complete", _I, [_P, C.POINTER(C.c_int)]),
    ("dcrt_tracer_acquire_film_clear_trigger", _I, [_P, C.POINTER(C.c_int)]),
    ("dcrt_tracer_clear_film", _I, [_P]),
    ("dcrt_tracer_accumulate_film", _I, [_P, C.POINTER(FilterParams)]),
    ("dcrt_tracer_read_film", _I, [_P, _FP]),
    ("dcrt_tracer_read_samples", _I, [_P, _FP, _FP]),
    ("dcrt_tracer_read_rng", _I, [_P, C.POINTER(C.c_uint32)]),
    ("dcrt_tracer_film_device_ptr", _I, [_P, C.POINTER(_P)]),
    ("dcrt_tracer_sample_device_ptrs", _I, [_P, C.POINTER(_P), C.POINTER(_P)]),
    ("dcrt_tracer_copy_film_device", _I, [_P, _P]),
    ("dcrt_tracer_add_film_device", _I, [_P, _P]),
    ("dcrt_tracer_prepare_images", _I, [_P, C.c_uint32]),
    ("dcrt_tracer_counters", _I, [_P, C.POINTER(RayStats)]),
    ("dcrt_tracer_set_instrumentation", _I, [_P, _I, _I]),
    ("dcrt_tracer_traversal_stats", _I, [_P, C.POINTER(TraversalStats)]),
    ("dcrt_tracer_reset_stats", _I, [_P]),
    ("dcrt_tracer_get_info", _I, [_P, C.POINTER(TracerInfo)]),
    ("dcrt_tracer_debug_ring_spills", _I, [_P, C.POINTER(C.c_uint64)]),
    ("dcrt_tracer_synchronize", _I, [_P]),
    ("dcrt_tracer_get_luts", _I, [_P, C.POINTER(BxDFLuts)]),
    ("dcrt_tracer_set_luts", _I, [_P, C.POINTER(BxDFLuts)]),
    ("dcrt_tracer_trace_rays", _I, [_P, C.POINTER(Ray), _U, C.POINTER(RayHit), _U]),
    ("dcrt_tracer_occluded", _I, [_P, C.POINTER(Ray), _U, C.POINTER(C.c_uint32), _U]),
    ("dcrt_tracer_trace_rays_device", _I, [_P, _P, _U, _P, _U]),
    ("dcrt_scene_get_postfx_params", _I, [_P, C.POINTER(PostFxParams)]),
    ("dcrt_srgb_encode_thresholds", _I, [_FP]),
    ("dcrt_tracer_resolve_image", _I, [_P, C.POINTER(PostFxParams), C.POINTER(C.c_uint8), _FP]),
    ("dcrt_write_bmp", _I, [C.c_char_p, _U, _U, C.POINTER(C.c_uint8)]),
    ("dcrt_device_math_eval", _I, [_P, _I, _FP, _U, _FP]),
]

_lib = None


class DCRTError(RuntimeError):
    pass


def load_library(path: os.PathLike | str | None = None):
    """Load libdcrt.so (built in-tree by __graft_entry__.build()). Raises if absent."""
    global _lib
    if _lib is not None:
        return _lib
    p = Path(path) if path else Path(os.environ.get("DCRT_LIB", LIB_PATH))
    if not p.exists():
        raise DCRTError(f"native library {p} is missing: run __graft_entry__.build() (no CPU fallback exists)")
    lib = C.CDLL(str(p))
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.dcrt_abi_version() != ABI_VERSION:
        raise DCRTError(f"{p}: ABI version {lib.dcrt_abi_version()}, this binding expects {ABI_VERSION}")
    _lib = lib
    return lib


def check(rc: int, what: str = "") -> None:
    if rc != DCRT_OK:
        lib = load_library()
        msg = lib.dcrt_last_error().decode(errors="replace")
        raise DCRTError(f"{what or 'dcrt call'} failed: {ERRORS.get(rc, rc)}: {msg}")


def f3(v) -> C.Array:
    return (C.c_float * 3)(*[float(x) for x in v])
