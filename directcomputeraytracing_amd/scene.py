"""Host scene (``CScene``, Source/Scene.h:67-224) over the C ABI.

Loading (OBJ, Mitsuba XML), BVH build (BVHAccel) and flattening run in the
native library; this class mirrors the reference's method names and exposes
zero-copy numpy views of the flattened Appendix-B buffers.
"""
from __future__ import annotations

import ctypes as C
from pathlib import Path

import numpy as np

from . import _abi
from ._abi import check, f3


class Scene:
    """CScene: LoadFromFile / Reset / lights / camera / film settings."""

    def __init__(self, resolution=(1920, 1080)):
        self._lib = _abi.load_library()
        h = C.c_void_p()
        check(self._lib.dcrt_scene_create(C.byref(h)), "dcrt_scene_create")
        self._h = h
        self.reset(*resolution)

    def close(self):
        if getattr(self, "_h", None):
            self._lib.dcrt_scene_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    @property
    def handle(self):
        return self._h

    # ---- CScene API -----------------------------------------------------
    def reset(self, width: int, height: int) -> None:            # Scene.cpp:626-660
        check(self._lib.dcrt_scene_reset(self._h, int(width), int(height)), "Reset")

    def load_from_file(self, path) -> None:                      # Scene.cpp:103-624
        check(self._lib.dcrt_scene_load_from_file(self._h, str(Path(path)).encode()), "LoadFromFile")

    def add_point_light(self, position, color) -> None:          # ImGui.cpp:322-331
        check(self._lib.dcrt_scene_add_punctual_light(self._h, f3(position), f3((0, 0, 0)), f3(color), 0), "AddPointLight")

    def add_directional_light(self, euler_angles, color) -> None:
        check(self._lib.dcrt_scene_add_punctual_light(self._h, f3((0, 0, 0)), f3(euler_angles), f3(color), 1),
              "AddDirectionalLight")

    def set_environment_light(self, color, cube: np.ndarray | None = None) -> None:
        if cube is None:
            check(self._lib.dcrt_scene_set_environment_light(self._h, f3(color), None, 0), "SetEnvironmentLight")
            return
        cube = np.ascontiguousarray(cube, dtype=np.float32)
        assert cube.ndim == 4 and cube.shape[0] == 6 and cube.shape[1] == cube.shape[2] and cube.shape[3] == 3
        self._env_cube = cube
        check(self._lib.dcrt_scene_set_environment_light(self._h, f3(color), cube.ctypes.data_as(_abi._FP),
                                                         cube.shape[1]), "SetEnvironmentLight")

    def set_camera(self, position, euler_angles=(0.0, 0.0, 0.0)) -> None:
        check(self._lib.dcrt_scene_set_camera(self._h, f3(position), f3(euler_angles)), "SetCamera")

    def set_lens(self, camera_type=1, fov_x=1.221730, focal_length=0.05, focal_distance=2.0, relative_aperture=8.0,
                 blade_count=7, aperture_rotation=0.0, film_size=(0.05333, 0.03)) -> None:
        fs = (C.c_float * 2)(*film_size)
        check(self._lib.dcrt_scene_set_lens(self._h, int(camera_type), fov_x, focal_length, focal_distance,
                                            relative_aperture, int(blade_count), aperture_rotation, fs), "SetLens")

    def set_max_bounce(self, n: int) -> None:
        check(self._lib.dcrt_scene_set_max_bounce(self._h, int(n)), "SetMaxBounce")

    def set_filter(self, kind=_abi.FILTER_BOX, radius=1.0, gaussian_alpha=1.5, mitchell_b=1 / 3, mitchell_c=1 / 3,
                   lanczos_tau=3) -> None:
        f = _abi.FilterParams(kind, radius, gaussian_alpha, mitchell_b, mitchell_c, lanczos_tau)
        check(self._lib.dcrt_scene_set_filter(self._h, C.byref(f)), "SetFilter")

    def filter_params(self) -> _abi.FilterParams:
        f = _abi.FilterParams()
        check(self._lib.dcrt_scene_get_filter(self._h, C.byref(f)), "GetFilter")
        return f

    def set_material(self, index, material_type, albedo=None, roughness=1.0, ior=None, k=None,
                     multiscattering=False, two_sided=False) -> None:
        check(self._lib.dcrt_scene_set_material(self._h, int(index), int(material_type),
                                                f3(albedo) if albedo is not None else None, float(roughness),
                                                f3(ior) if ior is not None else None,
                                                f3(k) if k is not None else None,
                                                int(multiscattering), int(two_sided)), "SetMaterial")

    def material_setting(self, index) -> _abi.MaterialSetting:   # SMaterial, Material.h:14-30
        m = _abi.MaterialSetting()
        check(self._lib.dcrt_scene_get_material_setting(self._h, int(index), C.byref(m)), "GetMaterialSetting")
        return m

    def set_multiscattering(self, index, enable: bool = True) -> None:   # ImGui.cpp:620-626
        check(self._lib.dcrt_scene_set_material_multiscattering(self._h, int(index), int(bool(enable))),
              "SetMultiscattering")

    def enable_multiscattering(self) -> list:
        """Tick the UI's "Multiscattering" box (ImGui.cpp:620-626) on every material that has
        it -- plastic, conductor, dielectric; both loaders leave it off
        (SceneXMLLoading.cpp:869). Returns the material indices changed."""
        changed = []
        for i in range(self.material_count):
            if self.material_setting(i).material_type in (_abi.MATERIAL_PLASTIC, _abi.MATERIAL_CONDUCTOR,
                                                          _abi.MATERIAL_DIELECTRIC):
                self.set_multiscattering(i, True)
                changed.append(i)
        return changed

    def settings(self) -> _abi.SceneSettings:
        s = _abi.SceneSettings()
        check(self._lib.dcrt_scene_get_settings(self._h, C.byref(s)), "GetSettings")
        return s

    def mesh_lights(self):
        """[(instance index in load order, (r, g, b))] -- SMeshLight, Scene.h:42-46."""
        out = []
        for i in range(self.settings().mesh_light_count):
            inst, col = C.c_uint32(), (C.c_float * 3)()
            check(self._lib.dcrt_scene_get_mesh_light(self._h, i, C.byref(inst), col))
            out.append((inst.value, tuple(col)))
        return out

    def punctual_lights(self):
        """[(position, euler angles, color, is_directional)] -- SPunctualLight, Scene.h:27-40."""
        out = []
        for i in range(self.settings().punctual_light_count):
            p, e, c, d = (C.c_float * 3)(), (C.c_float * 3)(), (C.c_float * 3)(), C.c_int()
            check(self._lib.dcrt_scene_get_punctual_light(self._h, i, p, e, c, C.byref(d)))
            out.append((tuple(p), tuple(e), tuple(c), bool(d.value)))
        return out

    def instance_material_overrides(self):
        """SMeshInstance::m_MaterialIdOverride per instance, load order."""
        _, ni = C.c_uint32(), C.c_uint32()
        check(self._lib.dcrt_scene_get_content_counts(self._h, C.byref(_), C.byref(ni)))
        out = []
        for j in range(ni.value):
            o = C.c_uint32()
            check(self._lib.dcrt_scene_get_instance_material_override(self._h, j, C.byref(o)))
            out.append(o.value)
        return out

    def set_material_opacity(self, index, opacity=1.0, opacity_texture_index=-1) -> None:   # ImGui.cpp:630-650
        check(self._lib.dcrt_scene_set_material_opacity(self._h, int(index), float(opacity), int(opacity_texture_index)),
              "SetMaterialOpacity")

    @property
    def features(self) -> int:
        """DCRT_FEATURE_* toggles (Scene.h:141-145); frame_params() carries them."""
        n = C.c_uint32()
        check(self._lib.dcrt_scene_get_features(self._h, C.byref(n)))
        return n.value

    @features.setter
    def features(self, value: int) -> None:
        check(self._lib.dcrt_scene_set_features(self._h, int(value)), "SetFeatures")

    @property
    def material_count(self) -> int:
        n = C.c_uint32()
        check(self._lib.dcrt_scene_get_material_count(self._h, C.byref(n)))
        return n.value

    @property
    def resolution(self):
        w, h = C.c_uint32(), C.c_uint32()
        check(self._lib.dcrt_scene_get_resolution(self._h, C.byref(w), C.byref(h)))
        return w.value, h.value

    def bvh_info(self):
        t, n, s = C.c_uint32(), C.c_uint32(), C.c_uint32()
        check(self._lib.dcrt_scene_get_bvh_info(self._h, C.byref(t), C.byref(n), C.byref(s)))
        return {"tlas_nodes": t.value, "total_nodes": n.value, "stack_size": s.value}

    def flat(self) -> _abi.FlatScene:
        f = _abi.FlatScene()
        check(self._lib.dcrt_scene_get_flat(self._h, C.byref(f)), "GetFlat")
        return f

    def postfx_params(self) -> _abi.PostFxParams:
        """Scene.h:181-185 defaults, EV100 from the camera (PostProcessing.cpp:39-42)."""
        p = _abi.PostFxParams()
        check(self._lib.dcrt_scene_get_postfx_params(self._h, C.byref(p)), "GetPostFxParams")
        return p

    def frame_params(self, frame_seed: int = 0) -> _abi.FrameParams:
        p = _abi.FrameParams()
        check(self._lib.dcrt_scene_get_frame_params(self._h, int(frame_seed), C.byref(p)), "GetFrameParams")
        return p

    def loaded_content(self):
        """Meshes and instances as loaded, before the BVH build reordered them (the inputs
        of Mesh::BuildBVH / BuildTLAS, Scene.cpp:160-215): ([{"vertices", "indices",
        "material_ids"}], [(mesh_index, (4, 3) transform)]), copies."""
        nm, ni = C.c_uint32(), C.c_uint32()
        check(self._lib.dcrt_scene_get_content_counts(self._h, C.byref(nm), C.byref(ni)))
        meshes = []
        for i in range(nm.value):
            m = _abi.ObjMesh()
            check(self._lib.dcrt_scene_get_loaded_mesh(self._h, i, C.byref(m)), "GetLoadedMesh")
            nv, nt = m.vertex_count, m.triangle_count
            meshes.append({
                "vertices": np.ctypeslib.as_array(C.cast(m.vertices, C.POINTER(C.c_float)), (nv * 11,)).reshape(nv, 11).copy(),
                "indices": np.ctypeslib.as_array(m.indices, (nt * 3,)).reshape(nt, 3).copy(),
                "material_ids": np.ctypeslib.as_array(m.material_ids, (nt,)).copy()})
        instances = []
        for j in range(ni.value):
            mesh = C.c_uint32()
            t = (C.c_float * 12)()
            check(self._lib.dcrt_scene_get_instance(self._h, j, C.byref(mesh), t))
            instances.append((mesh.value, np.array(t[:], np.float32).reshape(4, 3)))
        return meshes, instances

    # ---- numpy views of the flattened buffers (valid until the scene changes)
    def arrays(self) -> dict:
        f = self.flat()

        def view(ptr, count, dtype, cols=None):
            if count == 0 or not ptr:
                return np.zeros((0,) if cols is None else (0, cols), dtype=dtype)
            n = count * (cols or 1)
            a = np.ctypeslib.as_array(C.cast(ptr, C.POINTER(np.ctypeslib.as_ctypes_type(dtype))), shape=(n,))
            return a.reshape(-1, cols) if cols else a

        return {
            "vertices": view(f.vertices, f.vertex_count, np.float32, 11),
            "triangles": view(f.triangles, f.triangle_count, np.uint32, 3),
            "bvh_nodes": view(f.bvh_nodes, f.bvh_node_count, np.uint32, 8),
            "material_ids": view(f.material_ids, f.triangle_count, np.uint32),
            "instance_transforms": view(f.instance_transforms, f.instance_count * 2, np.float32, 12),
            "instance_flags": view(f.instance_flags, f.instance_count, np.uint32),
            "instance_material_overrides": view(f.instance_material_overrides, f.instance_count, np.uint32),
            "materials": view(f.materials, f.material_count, np.uint32, 13),
            "lights": view(f.lights, f.light_count, np.uint32, 7),
            "tlas_node_count": f.tlas_node_count,
            "stack_size": f.bvh_traversal_stack_size,
        }


def build_blas(vertices: np.ndarray, indices: np.ndarray) -> dict:
    """BVHAccel::BuildBLAS + PackBVH (BVHAccel.cpp:376-447) over one triangle mesh.

    ``vertices`` is an (N, 11) float32 array in the ``dcrt_vertex`` layout (or (N, 3)
    positions), ``indices`` (T, 3) uint32. Returns the packed nodes, the BVH-ordered
    index triples and the new->old triangle map, with the tree's depth and stack size."""
    lib = _abi.load_library()
    v = np.ascontiguousarray(vertices, np.float32)
    if v.ndim == 2 and v.shape[1] == 3:
        full = np.zeros((v.shape[0], 11), np.float32)
        full[:, :3] = v
        v = full
    idx = np.ascontiguousarray(indices, np.uint32).reshape(-1)
    n = idx.size // 3
    nodes = np.zeros((max(1, 2 * n), 8), np.uint32)
    reordered = np.zeros(idx.size, np.uint32)
    tri_map = np.zeros(n, np.uint32)
    count, depth, stack = C.c_uint32(), C.c_uint32(), C.c_uint32()
    check(lib.dcrt_bvh_build_blas(v.ctypes.data_as(C.POINTER(_abi.Vertex)), idx.ctypes.data_as(C.POINTER(C.c_uint32)), n,
                                  nodes.ctypes.data_as(C.POINTER(_abi.BVHNode)), C.byref(count),
                                  reordered.ctypes.data_as(C.POINTER(C.c_uint32)),
                                  tri_map.ctypes.data_as(C.POINTER(C.c_uint32)), C.byref(depth), C.byref(stack)),
          "BuildBLAS")
    return {"nodes": nodes[:count.value], "indices": reordered.reshape(-1, 3), "triangles": tri_map,
            "max_depth": depth.value, "max_stack_size": stack.value}


def load_obj_meshes(path, scene_layout: bool = True, material_index_base: int = 0) -> dict:
    """OBJ -> meshes before any BVH build (WavefrontOBJLoading.cpp:155-465) through
    ``dcrt_obj_load``: ``scene_layout`` gives the per-shape meshes of
    CScene::LoadFromWavefrontOBJFile (RH->LH), otherwise the one merged mesh the XML
    loader builds. Returns {"meshes": [{"vertices" (N, 11) f32, "indices" (T, 3) u32,
    "material_ids" (T,) u32}], "materials": [{"albedo", "ior", "roughness", "opacity",
    "albedo_texture_index", "opacity_texture_index"}]} (copies)."""
    lib = _abi.load_library()
    h = C.c_void_p()
    check(lib.dcrt_obj_load(str(path).encode(), _abi.OBJ_SCENE_LAYOUT if scene_layout else 0,
                            material_index_base, C.byref(h)), f"dcrt_obj_load({path})")
    try:
        n = C.c_uint32()
        check(lib.dcrt_obj_mesh_count(h, C.byref(n)))
        meshes = []
        for i in range(n.value):
            m = _abi.ObjMesh()
            check(lib.dcrt_obj_get_mesh(h, i, C.byref(m)))
            nv, nt = m.vertex_count, m.triangle_count
            verts = np.ctypeslib.as_array(C.cast(m.vertices, C.POINTER(C.c_float)), (nv * 11,)).reshape(nv, 11).copy() \
                if nv else np.zeros((0, 11), np.float32)
            idx = np.ctypeslib.as_array(m.indices, (nt * 3,)).reshape(nt, 3).copy() if nt else np.zeros((0, 3), np.uint32)
            mat = np.ctypeslib.as_array(m.material_ids, (nt,)).copy() if nt else np.zeros(0, np.uint32)
            meshes.append({"vertices": verts, "indices": idx, "material_ids": mat})
        check(lib.dcrt_obj_material_count(h, C.byref(n)))
        materials = []
        for i in range(n.value):
            mt = _abi.ObjMaterial()
            check(lib.dcrt_obj_get_material(h, i, C.byref(mt)))
            materials.append({"albedo": tuple(mt.albedo), "ior": mt.ior, "roughness": mt.roughness,
                              "opacity": mt.opacity, "albedo_texture_index": mt.albedo_texture_index,
                              "opacity_texture_index": mt.opacity_texture_index})
        return {"meshes": meshes, "materials": materials}
    finally:
        lib.dcrt_obj_free(h)
