// capi_scene.cpp -- extern "C" surface of the host scene (include/dcrt.h).
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <vector>
#include <exception>
#include <memory>
#include <string>

#include "../../../include/dcrt.h"
#include "scene.h"

namespace dcrt {
thread_local std::string g_lastError;
void SetLastError(const std::string& s) { g_lastError = s; }
}  // namespace dcrt

struct dcrt_scene {
    dcrt::CScene scene;
    // dcrt_scene_get_loaded_mesh's buffers, one pair per mesh, kept until the scene is
    // reset or loads more content (the pointers handed out stay valid until then)
    std::vector<std::vector<uint32_t>> loadedIndices, loadedMaterialIds;
    void DropLoadedBuffers() { loadedIndices.clear(); loadedMaterialIds.clear(); }
};

using dcrt::SetLastError;

#define DCRT_GUARD_BEGIN try {
#define DCRT_GUARD_END                                   \
    }                                                    \
    catch (const std::exception& e)                      \
    {                                                    \
        SetLastError(e.what());                          \
        return DCRT_E_INVALID_ARG;                       \
    }                                                    \
    catch (...)                                          \
    {                                                    \
        SetLastError("unknown C++ exception");           \
        return DCRT_E_INVALID_ARG;                       \
    }

extern "C" {

DCRT_API int dcrt_abi_version(void) { return DCRT_ABI_VERSION; }
DCRT_API const char* dcrt_version(void) { return "dcrt-mi355x 0.1.0 (gfx950)"; }
DCRT_API const char* dcrt_last_error(void) { return dcrt::g_lastError.c_str(); }

DCRT_API int dcrt_scene_create(dcrt_scene** out)
{
    if (!out) return DCRT_E_INVALID_ARG;
    DCRT_GUARD_BEGIN
    *out = new dcrt_scene();
    (*out)->scene.Reset(1920, 1080);
    return DCRT_OK;
    DCRT_GUARD_END
}

DCRT_API void dcrt_scene_destroy(dcrt_scene* s) { delete s; }

DCRT_API int dcrt_scene_reset(dcrt_scene* s, uint32_t w, uint32_t h)
{
    if (!s || !w || !h) return DCRT_E_INVALID_ARG;
    s->DropLoadedBuffers();
    s->scene.Reset(w, h);
    return DCRT_OK;
}

DCRT_API int dcrt_scene_load_from_file(dcrt_scene* s, const char* path)
{
    if (!s || !path) return DCRT_E_INVALID_ARG;
    DCRT_GUARD_BEGIN
    SetLastError("");
    s->DropLoadedBuffers();
    if (!s->scene.LoadFromFile(path)) {
        const std::string detail = dcrt_last_error();
        SetLastError(std::string("failed to load scene ") + path + (detail.empty() ? "" : ": " + detail));
        return DCRT_E_IO;
    }
    return DCRT_OK;
    DCRT_GUARD_END
}

DCRT_API int dcrt_scene_add_punctual_light(dcrt_scene* s, const float position[3], const float euler[3], const float color[3], int is_directional)
{
    if (!s || !position || !euler || !color) return DCRT_E_INVALID_ARG;
    if (s->scene.GetLightCount() >= DCRT_MAX_LIGHT_COUNT) return DCRT_E_LIMIT;
    dcrt::SPunctualLight l;
    l.position = dcrt::Float3(position[0], position[1], position[2]);
    l.eulerAngles = dcrt::Float3(euler[0], euler[1], euler[2]);
    l.color = dcrt::Float3(color[0], color[1], color[2]);
    l.isDirectional = is_directional != 0;
    s->scene.punctualLights.push_back(l);
    s->scene.Flatten();
    return DCRT_OK;
}

DCRT_API int dcrt_scene_set_environment_light(dcrt_scene* s, const float color[3], const float* cube, uint32_t cube_size)
{
    if (!s || !color) return DCRT_E_INVALID_ARG;
    s->scene.hasEnvironmentLight = true;
    s->scene.environmentLight.color = dcrt::Float3(color[0], color[1], color[2]);
    if (cube && cube_size) {
        s->scene.environmentLight.cubeSize = cube_size;
        s->scene.environmentLight.cubeRGB.assign(cube, cube + (size_t)6 * cube_size * cube_size * 3);
    } else {
        s->scene.environmentLight.cubeSize = 0;
        s->scene.environmentLight.cubeRGB.clear();
    }
    s->scene.Flatten();
    return DCRT_OK;
}

DCRT_API int dcrt_scene_set_camera(dcrt_scene* s, const float position[3], const float euler[3])
{
    if (!s || !position || !euler) return DCRT_E_INVALID_ARG;
    s->scene.camera.position = dcrt::Float3(position[0], position[1], position[2]);
    s->scene.camera.eulerAngles = dcrt::Float3(euler[0], euler[1], euler[2]);
    return DCRT_OK;
}

DCRT_API int dcrt_scene_set_lens(dcrt_scene* s, int camera_type, float fov_x, float focal_length, float focal_distance,
                                 float relative_aperture, uint32_t blade_count, float aperture_rotation, const float film_size[2])
{
    if (!s || (camera_type != 0 && camera_type != 1)) return DCRT_E_INVALID_ARG;
    s->scene.cameraType = (dcrt::ECameraType)camera_type;
    s->scene.fovX = fov_x;
    s->scene.focalLength = focal_length;
    s->scene.focalDistance = focal_distance;
    s->scene.relativeAperture = relative_aperture;
    s->scene.apertureBladeCount = blade_count;
    s->scene.apertureRotation = aperture_rotation;
    if (film_size) s->scene.filmSize = { film_size[0], film_size[1] };
    return DCRT_OK;
}

DCRT_API int dcrt_scene_set_max_bounce(dcrt_scene* s, uint32_t max_bounce)
{
    if (!s || max_bounce > DCRT_MAX_RAY_BOUNCE) return DCRT_E_INVALID_ARG;
    s->scene.maxBounceCount = max_bounce;
    return DCRT_OK;
}

DCRT_API int dcrt_scene_set_filter(dcrt_scene* s, const dcrt_filter_params* f)
{
    if (!s || !f || f->filter > DCRT_FILTER_LANCZOS || !(f->radius >= 0.0f)) return DCRT_E_INVALID_ARG;
    s->scene.filter = (dcrt::EFilter)f->filter;
    s->scene.filterRadius = f->radius;
    s->scene.gaussianFilterAlpha = f->gaussian_alpha;
    s->scene.mitchellB = f->mitchell_b;
    s->scene.mitchellC = f->mitchell_c;
    s->scene.lanczosSincTau = f->lanczos_tau ? f->lanczos_tau : 3;
    return DCRT_OK;
}

DCRT_API int dcrt_scene_get_filter(const dcrt_scene* s, dcrt_filter_params* out)
{
    if (!s || !out) return DCRT_E_INVALID_ARG;
    *out = s->scene.GetFilterParams();
    return DCRT_OK;
}

DCRT_API int dcrt_scene_get_resolution(const dcrt_scene* s, uint32_t* w, uint32_t* h)
{
    if (!s || !w || !h) return DCRT_E_INVALID_ARG;
    *w = s->scene.resolutionWidth;
    *h = s->scene.resolutionHeight;
    return DCRT_OK;
}

DCRT_API int dcrt_scene_get_material_count(const dcrt_scene* s, uint32_t* out)
{
    if (!s || !out) return DCRT_E_INVALID_ARG;
    *out = (uint32_t)s->scene.materials.size();
    return DCRT_OK;
}

// Material edits: mesh OPAQUE flags (Scene.cpp:57-80) and the flattened buffers
// (instance flags, Scene.cpp:785-800) follow the materials.
static void RefreshMaterials(dcrt_scene* s)
{
    if (!s->scene.hasValidScene) return;
    for (size_t i = 0; i < s->scene.meshes.size(); ++i) {
        bool opaque = true;
        for (uint32_t id : s->scene.meshes[i].materialIds) opaque = opaque && s->scene.materials[id].IsOpaque();
        s->scene.meshOpaque[i] = opaque;
    }
    s->scene.Flatten();
}

DCRT_API int dcrt_scene_set_material(dcrt_scene* s, uint32_t index, int type, const float albedo[3], float roughness,
                                     const float ior[3], const float k[3], int multiscattering, int two_sided)
{
    if (!s || index >= s->scene.materials.size() || type < 0 || type > 4) return DCRT_E_INVALID_ARG;
    dcrt::SMaterial& m = s->scene.materials[index];
    m.type = (dcrt::EMaterialType)type;
    if (albedo) m.albedo = dcrt::Float3(albedo[0], albedo[1], albedo[2]);
    m.roughness = roughness;
    if (ior) m.ior = dcrt::Float3(ior[0], ior[1], ior[2]);
    if (k) m.k = dcrt::Float3(k[0], k[1], k[2]);
    m.multiscattering = multiscattering != 0;
    m.isTwoSided = two_sided != 0;
    RefreshMaterials(s);
    return DCRT_OK;
}

DCRT_API int dcrt_scene_get_material_setting(const dcrt_scene* s, uint32_t index, dcrt_material_setting* out)
{
    if (!s || !out || index >= s->scene.materials.size()) return DCRT_E_INVALID_ARG;
    const dcrt::SMaterial& m = s->scene.materials[index];
    *out = dcrt_material_setting{};
    out->albedo[0] = m.albedo.x; out->albedo[1] = m.albedo.y; out->albedo[2] = m.albedo.z;
    out->roughness = m.roughness;
    out->ior[0] = m.ior.x; out->ior[1] = m.ior.y; out->ior[2] = m.ior.z;
    out->opacity = m.opacity;
    out->k[0] = m.k.x; out->k[1] = m.k.y; out->k[2] = m.k.z;
    out->tiling[0] = m.tiling.x; out->tiling[1] = m.tiling.y;
    out->material_type = (uint32_t)m.type;
    out->albedo_texture_index = m.albedoTextureIndex;
    out->opacity_texture_index = m.opacityTextureIndex;
    out->internal_scattering_mode = m.internalScatteringMode;
    out->multiscattering = m.multiscattering;
    out->is_two_sided = m.isTwoSided;
    out->has_roughness_texture = m.hasRoughnessTexture;
    return DCRT_OK;
}

DCRT_API int dcrt_scene_set_material_multiscattering(dcrt_scene* s, uint32_t index, int enable)
{
    if (!s || index >= s->scene.materials.size()) return DCRT_E_INVALID_ARG;
    dcrt::SMaterial& m = s->scene.materials[index];
    if (m.type == dcrt::EMaterialType::Diffuse || m.type == dcrt::EMaterialType::ThinDielectric) {
        SetLastError("multiscattering applies to plastic, conductor and dielectric materials (ImGui.cpp:620)");
        return DCRT_E_INVALID_ARG;
    }
    m.multiscattering = enable != 0;
    RefreshMaterials(s);
    return DCRT_OK;
}

DCRT_API int dcrt_scene_set_material_opacity(dcrt_scene* s, uint32_t index, float opacity, int32_t opacity_texture_index)
{
    if (!s || index >= s->scene.materials.size()) return DCRT_E_INVALID_ARG;
    if (opacity_texture_index < -1 || (opacity_texture_index >= 0 && (size_t)opacity_texture_index >= s->scene.textures.size()))
        return DCRT_E_INVALID_ARG;
    dcrt::SMaterial& m = s->scene.materials[index];
    m.opacity = opacity;
    m.opacityTextureIndex = opacity_texture_index;
    RefreshMaterials(s);
    return DCRT_OK;
}

DCRT_API int dcrt_scene_set_features(dcrt_scene* s, uint32_t features)
{
    const uint32_t known = DCRT_FEATURE_GGX_SAMPLE_VNDF | DCRT_FEATURE_NO_FRONT_TO_BACK | DCRT_FEATURE_LIGHT_VISIBLE |
                           DCRT_FEATURE_WATERTIGHT | DCRT_FEATURE_ALLOW_ANYHIT;
    if (!s || (features & ~known)) return DCRT_E_INVALID_ARG;
    s->scene.features = features;
    return DCRT_OK;
}

DCRT_API int dcrt_scene_get_features(const dcrt_scene* s, uint32_t* out)
{
    if (!s || !out) return DCRT_E_INVALID_ARG;
    *out = s->scene.features;
    return DCRT_OK;
}

DCRT_API int dcrt_scene_get_flat(dcrt_scene* s, dcrt_flat_scene* out)
{
    if (!s || !out) return DCRT_E_INVALID_ARG;
    if (!s->scene.hasValidScene) { SetLastError("scene has no content"); return DCRT_E_NO_SCENE; }
    *out = s->scene.GetFlat();
    return DCRT_OK;
}

DCRT_API int dcrt_scene_get_frame_params(const dcrt_scene* s, uint32_t seed, dcrt_frame_params* out)
{
    if (!s || !out) return DCRT_E_INVALID_ARG;
    *out = s->scene.GetFrameParams(seed);
    return DCRT_OK;
}

DCRT_API int dcrt_scene_get_bvh_info(const dcrt_scene* s, uint32_t* tlas_nodes, uint32_t* total_nodes, uint32_t* max_stack)
{
    if (!s) return DCRT_E_INVALID_ARG;
    uint32_t total = (uint32_t)s->scene.tlas.size();
    for (const dcrt::Mesh& m : s->scene.meshes) total += (uint32_t)m.bvhNodes.size();
    if (tlas_nodes) *tlas_nodes = (uint32_t)s->scene.tlas.size();
    if (total_nodes) *total_nodes = total;
    if (max_stack) *max_stack = s->scene.bvhTraversalStackSize;
    return DCRT_OK;
}

DCRT_API int dcrt_bvh_build_blas(const dcrt_vertex* vertices, const uint32_t* indices, uint32_t triangle_count, dcrt_bvh_node* out_nodes,
                                 uint32_t* out_node_count, uint32_t* out_reordered_indices, uint32_t* out_reordered_triangles,
                                 uint32_t* out_max_depth, uint32_t* out_max_stack_size)
{
    if (!vertices || !indices || !out_nodes || !out_node_count || !out_reordered_indices || !out_reordered_triangles || !triangle_count)
        return DCRT_E_INVALID_ARG;
    DCRT_GUARD_BEGIN
    dcrt::bvh::BuildResult r;
    dcrt::bvh::BuildBLAS(vertices, indices, triangle_count, out_reordered_indices, out_reordered_triangles, &r);
    dcrt::bvh::PackBVH(r.nodes.data(), (uint32_t)r.nodes.size(), true, out_nodes);
    *out_node_count = (uint32_t)r.nodes.size();
    if (out_max_depth) *out_max_depth = r.maxDepth;
    if (out_max_stack_size) *out_max_stack_size = r.maxStackSize;
    return DCRT_OK;
    DCRT_GUARD_END
}

DCRT_API int dcrt_scene_get_content_counts(const dcrt_scene* s, uint32_t* meshes, uint32_t* instances)
{
    if (!s || !meshes || !instances) return DCRT_E_INVALID_ARG;
    *meshes = (uint32_t)s->scene.meshes.size();
    *instances = (uint32_t)s->scene.meshInstances.size();
    return DCRT_OK;
}

DCRT_API int dcrt_scene_get_loaded_mesh(dcrt_scene* s, uint32_t index, dcrt_obj_mesh* out)
{
    if (!s || !out || index >= s->scene.meshes.size()) return DCRT_E_INVALID_ARG;
    DCRT_GUARD_BEGIN
    const dcrt::Mesh& m = s->scene.meshes[index];
    const uint32_t n = m.GetTriangleCount();
    if (m.bvhTriangleOrder.size() != n) { SetLastError("mesh has no BVH yet"); return DCRT_E_NO_SCENE; }
    if (s->loadedIndices.size() != s->scene.meshes.size()) {
        s->loadedIndices.assign(s->scene.meshes.size(), {});
        s->loadedMaterialIds.assign(s->scene.meshes.size(), {});
    }
    std::vector<uint32_t>& idx = s->loadedIndices[index];
    std::vector<uint32_t>& ids = s->loadedMaterialIds[index];
    if (idx.size() != (size_t)n * 3 || ids.size() != n) {
        idx.assign((size_t)n * 3, 0);
        ids.assign(n, 0);
        for (uint32_t t = 0; t < n; ++t) {   // BVH position t holds load-order triangle order[t]
            const uint32_t src = m.bvhTriangleOrder[t];
            for (int k = 0; k < 3; ++k) idx[(size_t)src * 3 + k] = m.indices[(size_t)t * 3 + k];
            ids[src] = m.materialIds[t];
        }
    }
    out->vertices = m.vertices.data();
    out->vertex_count = (uint32_t)m.vertices.size();
    out->indices = idx.data();
    out->material_ids = ids.data();
    out->triangle_count = n;
    return DCRT_OK;
    DCRT_GUARD_END
}

DCRT_API int dcrt_scene_get_instance(const dcrt_scene* s, uint32_t index, uint32_t* mesh, float transform[12])
{
    if (!s || !mesh || !transform || index >= s->scene.meshInstances.size()) return DCRT_E_INVALID_ARG;
    *mesh = s->scene.meshInstances[index].meshIndex;
    const dcrt::Float4x3& t = s->scene.instanceTransforms[index];
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 3; ++c) transform[r * 3 + c] = t.m[r][c];
    return DCRT_OK;
}

DCRT_API int dcrt_scene_get_settings(const dcrt_scene* s, dcrt_scene_settings* out)
{
    if (!s || !out) return DCRT_E_INVALID_ARG;
    const dcrt::CScene& sc = s->scene;
    *out = dcrt_scene_settings{};
    out->resolution[0] = sc.resolutionWidth;
    out->resolution[1] = sc.resolutionHeight;
    out->max_bounce_count = sc.maxBounceCount;
    out->camera_type = (uint32_t)sc.cameraType;
    out->fov_x = sc.fovX;
    out->focal_length = sc.focalLength;
    out->focal_distance = sc.focalDistance;
    out->relative_aperture = sc.relativeAperture;
    out->aperture_blade_count = sc.apertureBladeCount;
    out->aperture_rotation = sc.apertureRotation;
    out->film_size[0] = sc.filmSize.x;
    out->film_size[1] = sc.filmSize.y;
    const dcrt::Float3 p = sc.camera.position, e = sc.camera.eulerAngles;
    out->camera_position[0] = p.x; out->camera_position[1] = p.y; out->camera_position[2] = p.z;
    out->camera_euler_angles[0] = e.x; out->camera_euler_angles[1] = e.y; out->camera_euler_angles[2] = e.z;
    out->features = sc.features;
    out->has_environment_light = sc.hasEnvironmentLight;
    const dcrt::Float3 c = sc.environmentLight.color;
    out->environment_color[0] = c.x; out->environment_color[1] = c.y; out->environment_color[2] = c.z;
    out->env_cube_rgb = sc.environmentLight.cubeSize ? sc.environmentLight.cubeRGB.data() : nullptr;
    out->env_cube_size = sc.environmentLight.cubeSize;
    out->mesh_light_count = (uint32_t)sc.meshLights.size();
    out->punctual_light_count = (uint32_t)sc.punctualLights.size();
    out->material_count = (uint32_t)sc.materials.size();
    out->texture_count = (uint32_t)sc.textures.size();
    return DCRT_OK;
}

DCRT_API int dcrt_scene_get_mesh_light(const dcrt_scene* s, uint32_t index, uint32_t* instance, float color[3])
{
    if (!s || !instance || !color || index >= s->scene.meshLights.size()) return DCRT_E_INVALID_ARG;
    const dcrt::SMeshLight& l = s->scene.meshLights[index];
    *instance = l.instanceIndex;
    color[0] = l.color.x; color[1] = l.color.y; color[2] = l.color.z;
    return DCRT_OK;
}

DCRT_API int dcrt_scene_get_punctual_light(const dcrt_scene* s, uint32_t index, float position[3], float euler[3],
                                           float color[3], int* is_directional)
{
    if (!s || !position || !euler || !color || !is_directional || index >= s->scene.punctualLights.size())
        return DCRT_E_INVALID_ARG;
    const dcrt::SPunctualLight& l = s->scene.punctualLights[index];
    position[0] = l.position.x; position[1] = l.position.y; position[2] = l.position.z;
    euler[0] = l.eulerAngles.x; euler[1] = l.eulerAngles.y; euler[2] = l.eulerAngles.z;
    color[0] = l.color.x; color[1] = l.color.y; color[2] = l.color.z;
    *is_directional = l.isDirectional;
    return DCRT_OK;
}

DCRT_API int dcrt_scene_get_instance_material_override(const dcrt_scene* s, uint32_t index, uint32_t* out)
{
    if (!s || !out || index >= s->scene.meshInstances.size()) return DCRT_E_INVALID_ARG;
    *out = s->scene.meshInstances[index].materialIdOverride;
    return DCRT_OK;
}

// ---- OBJ meshes before the BVH build (WavefrontOBJLoading.cpp:155-263,374-465)
struct dcrt_obj_meshes {
    std::vector<dcrt::Mesh> meshes;
    std::vector<dcrt::SMaterial> materials;
};

DCRT_API int dcrt_obj_load(const char* path, uint32_t flags, uint32_t material_index_base, dcrt_obj_meshes** out)
{
    if (!path || !out) return DCRT_E_INVALID_ARG;
    DCRT_GUARD_BEGIN
    std::unique_ptr<dcrt_obj_meshes> r(new dcrt_obj_meshes());
    dcrt::ObjData data;
    std::string err;
    if (!dcrt::ParseObjFile(path, &data, &err)) {
        SetLastError(err);
        return DCRT_E_IO;
    }
    dcrt::SMeshProcessingParams params;
    params.changeWindingOrder = true;
    params.flipTexcoordV = true;
    if (flags & DCRT_OBJ_SCENE_LAYOUT) {
        params.applyTransform = true;
        params.transform.m[0][0] = -1.0f;
        for (size_t s = 0; s < data.shapes.size(); ++s) {
            r->meshes.emplace_back();
            params.materialIndexBase = material_index_base;
            if (!dcrt::CreateMeshFromObjData(data, &data.shapes[s], 1, params, &r->meshes.back())) {
                SetLastError("mesh creation failed");
                return DCRT_E_IO;
            }
        }
    } else {
        params.materialIndexBase = material_index_base;
        r->meshes.emplace_back();
        if (!dcrt::CreateMeshFromObjData(data, data.shapes.data(), (uint32_t)data.shapes.size(), params, &r->meshes.back())) {
            SetLastError("mesh creation failed");
            return DCRT_E_IO;
        }
    }
    std::vector<std::string> textureNames;
    dcrt::TranslateObjMaterials(data, 0, &r->materials, &textureNames);
    *out = r.release();
    return DCRT_OK;
    DCRT_GUARD_END
}

DCRT_API int dcrt_obj_mesh_count(const dcrt_obj_meshes* m, uint32_t* out)
{
    if (!m || !out) return DCRT_E_INVALID_ARG;
    *out = (uint32_t)m->meshes.size();
    return DCRT_OK;
}

DCRT_API int dcrt_obj_get_mesh(const dcrt_obj_meshes* m, uint32_t index, dcrt_obj_mesh* out)
{
    if (!m || !out || index >= m->meshes.size()) return DCRT_E_INVALID_ARG;
    const dcrt::Mesh& mesh = m->meshes[index];
    out->vertices = mesh.vertices.data();
    out->vertex_count = (uint32_t)mesh.vertices.size();
    out->indices = mesh.indices.data();
    out->material_ids = mesh.materialIds.data();
    out->triangle_count = mesh.GetTriangleCount();
    return DCRT_OK;
}

DCRT_API int dcrt_obj_material_count(const dcrt_obj_meshes* m, uint32_t* out)
{
    if (!m || !out) return DCRT_E_INVALID_ARG;
    *out = (uint32_t)m->materials.size();
    return DCRT_OK;
}

DCRT_API int dcrt_obj_get_material(const dcrt_obj_meshes* m, uint32_t index, dcrt_obj_material* out)
{
    if (!m || !out || index >= m->materials.size()) return DCRT_E_INVALID_ARG;
    const dcrt::SMaterial& s = m->materials[index];
    out->albedo[0] = s.albedo.x; out->albedo[1] = s.albedo.y; out->albedo[2] = s.albedo.z;
    out->ior = s.ior.x;
    out->roughness = s.roughness;
    out->opacity = s.opacity;
    out->albedo_texture_index = s.albedoTextureIndex;
    out->opacity_texture_index = s.opacityTextureIndex;
    return DCRT_OK;
}

DCRT_API void dcrt_obj_free(dcrt_obj_meshes* m) { delete m; }

DCRT_API int dcrt_xml_dump_tree(const char* path, char* out, uint32_t capacity, uint32_t* out_length)
{
    if (!path || !out_length) return DCRT_E_INVALID_ARG;
    DCRT_GUARD_BEGIN
    std::string dump;
    if (!dcrt::DumpXmlTree(path, &dump)) return DCRT_E_IO;
    *out_length = (uint32_t)dump.size();
    if (out && capacity) {
        const size_t n = std::min<size_t>(dump.size(), capacity);
        std::memcpy(out, dump.data(), n);
    }
    return dump.size() <= capacity ? DCRT_OK : DCRT_E_LIMIT;
    DCRT_GUARD_END
}

}  // extern "C"

extern "C" {

DCRT_API int dcrt_scene_get_postfx_params(const dcrt_scene* s, dcrt_postfx_params* out)
{
    if (!s || !out) return DCRT_E_INVALID_ARG;
    const dcrt::CScene& sc = s->scene;
    out->enabled = 1;
    out->auto_exposure = 1;
    // CalculateEV100 (PostProcessing.cpp:39-42)
    out->ev100 = std::log2(sc.relativeAperture * sc.relativeAperture / sc.shutterTime * 100 / sc.iso);
    out->luminance_white = 1.0f;
    return DCRT_OK;
}

DCRT_API int dcrt_srgb_encode_thresholds(float out[255])
{
    if (!out) return DCRT_E_INVALID_ARG;
    for (int k = 0; k < 255; ++k) {
        const double c = (k + 0.5) / 255.0;
        const double lin = c <= 0.04045 ? c / 12.92 : std::pow((c + 0.055) / 1.055, 2.4);
        out[k] = (float)lin;
    }
    return DCRT_OK;
}

DCRT_API int dcrt_write_bmp(const char* path, uint32_t w, uint32_t h, const uint8_t* rgba)
{
    if (!path || !rgba || !w || !h) return DCRT_E_INVALID_ARG;
    const uint32_t stride = (w * 3 + 3) & ~3u;
    const uint32_t imageSize = stride * h, fileSize = 54 + imageSize;
    std::vector<uint8_t> buf(fileSize, 0);
    auto put32 = [&](size_t o, uint32_t v) { for (int i = 0; i < 4; ++i) buf[o + i] = (uint8_t)(v >> (8 * i)); };
    auto put16 = [&](size_t o, uint16_t v) { buf[o] = (uint8_t)v; buf[o + 1] = (uint8_t)(v >> 8); };
    buf[0] = 'B'; buf[1] = 'M';
    put32(2, fileSize); put32(10, 54);
    put32(14, 40); put32(18, w); put32(22, h); put16(26, 1); put16(28, 24);
    put32(34, imageSize); put32(38, 2835); put32(42, 2835);
    for (uint32_t y = 0; y < h; ++y) {
        const uint8_t* src = rgba + (size_t)(h - 1 - y) * w * 4;    // bottom-up rows
        uint8_t* dst = buf.data() + 54 + (size_t)y * stride;
        for (uint32_t x = 0; x < w; ++x) {
            dst[x * 3 + 0] = src[x * 4 + 2];
            dst[x * 3 + 1] = src[x * 4 + 1];
            dst[x * 3 + 2] = src[x * 4 + 0];
        }
    }
    FILE* f = std::fopen(path, "wb");
    if (!f) { SetLastError(std::string("cannot write ") + path); return DCRT_E_IO; }
    const bool ok = std::fwrite(buf.data(), 1, buf.size(), f) == buf.size();
    std::fclose(f);
    if (!ok) { SetLastError(std::string("short write ") + path); return DCRT_E_IO; }
    return DCRT_OK;
}

}  // extern "C"
