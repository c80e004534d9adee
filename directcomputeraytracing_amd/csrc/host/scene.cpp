// scene.cpp -- CScene restated for the MI355X tracer (Source/Scene.cpp,
// Mesh.cpp, Camera.cpp). Produces exactly the buffers Scene.cpp:273-608 and
// UpdateLight/Material/InstanceFlagsGPUData (Scene.cpp:672-807) upload.
#include "scene.h"

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>

namespace dcrt {

void SetLastError(const std::string& s);   // (capi_scene.cpp)

void GetDefaultMaterial(SMaterial* m)
{
    *m = SMaterial();
    m->albedo = Float3(1.0f, 0.0f, 1.0f);
    m->roughness = 1.0f;
    m->ior = Float3(1.0f, 1.0f, 1.0f);
    m->opacity = 1.0f;
    m->k = Float3(1.0f, 1.0f, 1.0f);
    m->tiling = { 1.0f, 1.0f };
    m->type = EMaterialType::Diffuse;
    m->albedoTextureIndex = -1;
    m->opacityTextureIndex = -1;
    m->multiscattering = false;
    m->isTwoSided = false;
    m->hasRoughnessTexture = false;
    m->internalScatteringMode = DCRT_INTERNAL_SCATTERING_MULTIPLE;
    m->name = "DefaultMaterial";
}

// ---------------------------------------------------------------- Mesh
void Mesh::BuildBVH(std::vector<uint32_t>* reordered)
{
    std::vector<uint32_t> srcIndices = indices;
    reordered->resize(GetTriangleCount());
    bvh::BuildResult result;
    bvh::BuildBLAS(vertices.data(), srcIndices.data(), GetTriangleCount(), indices.data(), reordered->data(), &result);
    bvhNodes = std::move(result.nodes);
    bvhMaxDepth = result.maxDepth;
    bvhMaxStackSize = result.maxStackSize;
    std::vector<uint32_t> ids = materialIds;
    for (size_t i = 0; i < ids.size(); ++i) materialIds[i] = ids[(*reordered)[i]];
    bvhTriangleOrder = *reordered;
}

bool Mesh::GenerateRectangle(uint32_t materialId, bool applyTransform, const Float4x4& transform)
{
    static const dcrt_vertex kQuad[4] = {
        { { 1.0f, 1.0f, 0.0f }, { 0.0f, 0.0f, 1.0f }, { 1.0f, 0.0f, 0.0f }, { 1.0f, 1.0f } },
        { { 1.0f, -1.0f, 0.0f }, { 0.0f, 0.0f, 1.0f }, { 1.0f, 0.0f, 0.0f }, { 1.0f, 0.0f } },
        { { -1.0f, -1.0f, 0.0f }, { 0.0f, 0.0f, 1.0f }, { 1.0f, 0.0f, 0.0f }, { 0.0f, 0.0f } },
        { { -1.0f, 1.0f, 0.0f }, { 0.0f, 0.0f, 1.0f }, { 1.0f, 0.0f, 0.0f }, { 0.0f, 1.0f } },
    };
    static const uint32_t kIdx[6] = { 0, 1, 3, 1, 2, 3 };
    const uint32_t base = (uint32_t)vertices.size();
    const Float4x4 normalTransform = Transpose(Inverse(transform));
    for (const dcrt_vertex& src : kQuad) {
        dcrt_vertex v = src;
        v.texcoord[0] = 0.0f;   // Mesh.cpp:31-36 never copies the texcoord (value-initialised)
        v.texcoord[1] = 0.0f;
        // Mesh.cpp:28-38 always transforms (identity when applyTransform is false)
        const Float4x4& M = applyTransform ? transform : Float4x4::Identity();
        const Float4x4& N = applyTransform ? normalTransform : Float4x4::Identity();
        Float3 p = TransformPoint(Float3(v.position[0], v.position[1], v.position[2]), M);
        Float3 n = TransformNormal(Float3(v.normal[0], v.normal[1], v.normal[2]), N);
        Float3 t = TransformNormal(Float3(v.tangent[0], v.tangent[1], v.tangent[2]), N);
        v.position[0] = p.x; v.position[1] = p.y; v.position[2] = p.z;
        v.normal[0] = n.x; v.normal[1] = n.y; v.normal[2] = n.z;
        v.tangent[0] = t.x; v.tangent[1] = t.y; v.tangent[2] = t.z;
        vertices.push_back(v);
    }
    for (uint32_t i : kIdx) indices.push_back(base + i);
    materialIds.push_back(materialId);
    materialIds.push_back(materialId);
    return true;
}

// ---------------------------------------------------------------- Camera / lights
Float4x4 Camera::GetTransformMatrix() const
{
    Float4x4 m = RotationRollPitchYaw(eulerAngles.x, eulerAngles.y, eulerAngles.z);
    m.m[3][0] = position.x;
    m.m[3][1] = position.y;
    m.m[3][2] = position.z;
    return m;
}

Float3 SPunctualLight::CalculateDirection() const
{
    const Float4x4 m = RotationRollPitchYaw(eulerAngles.x, eulerAngles.y, eulerAngles.z);
    return TransformPoint(Float3(1.0f, 0.0f, 0.0f), m);
}

void SPunctualLight::SetEulerAnglesFromDirection(const Float3& direction)
{
    const Float3 initial(1.0f, 0.0f, 0.0f);
    Float3 axis = Cross(initial, direction);
    const float axisLength = Length(axis);
    const float dot = Dot(direction, initial);
    if (axisLength < 1e-7f) {
        eulerAngles = dot >= 0.0f ? Float3(0.0f, 0.0f, 0.0f) : Float3(0.0f, 3.14159265358979f, 0.0f);
        return;
    }
    // XMVectorDivide(axis, axisLength): a division per component (Scene.cpp:937)
    axis = Float3(axis.x / axisLength, axis.y / axisLength, axis.z / axisLength);
    const float angle = (float)std::acos((double)dot);
    // XMMatrixRotationAxis: XMVector3Normalize, then XMMatrixRotationNormal (XMScalarSinCos)
    const Float4x4 R = RotationNormal(Normalize3(axis), angle);
    eulerAngles = MatrixRotationToRollPitchYaw(R);
}

// ---------------------------------------------------------------- CScene
void CScene::Reset(uint32_t w, uint32_t h)
{
    resolutionWidth = w;
    resolutionHeight = h;
    maxBounceCount = 2;
    filmSize = { 0.05333f, 0.03f };
    cameraType = ECameraType::ThinLens;
    fovX = 1.221730f;
    focalLength = 0.05f;
    focalDistance = 2.0f;
    relativeAperture = 8.0f;
    apertureBladeCount = 7;
    apertureRotation = 0.0f;
    shutterTime = 1.0f;
    iso = 100.0f;
    filterRadius = 1.0f;
    camera = Camera();
    meshes.clear();
    meshInstances.clear();
    meshOpaque.clear();
    hasEnvironmentLight = false;
    environmentLight = SEnvironmentLight();
    punctualLights.clear();
    meshLights.clear();
    materials.clear();
    tlas.clear();
    originalInstanceIndices.clear();
    reorderedInstanceIndices.clear();
    instanceTransforms.clear();
    textures.clear();
    hasValidScene = false;
}

float CScene::CalculateFilmDistance() const
{
    return cameraType == ECameraType::PinHole ? 0.5f * filmSize.x / std::max(std::tan(0.5f * fovX), 0.0001f)
                                              : (focalLength * focalDistance) / (focalLength + focalDistance);
}

float CScene::CalculateApertureDiameter() const
{
    return cameraType == ECameraType::PinHole ? 0.0f : focalLength / relativeAperture;
}

bool CScene::LoadFromFile(const std::string& path)
{
    if (path.empty()) return false;
    const size_t meshIndexBase = meshes.size();
    {
        const size_t dot = path.find_last_of('.');
        const std::string ext = dot == std::string::npos ? std::string() : path.substr(dot);
        const bool isXml = ext == ".xml" || ext == ".XML";
        if (!(isXml ? LoadFromXMLFile(path) : LoadFromWavefrontOBJFile(path))) return false;
    }
    // Assign default material (Scene.cpp:126-160)
    {
        uint32_t defaultIndex = kInvalidMaterialId;
        for (size_t i = meshIndexBase; i < meshes.size(); ++i)
            for (uint32_t& id : meshes[i].materialIds)
                if (id == kInvalidMaterialId) {
                    if (defaultIndex == kInvalidMaterialId) defaultIndex = (uint32_t)materials.size();
                    id = defaultIndex;
                }
        if (defaultIndex != kInvalidMaterialId) {
            SMaterial m;
            GetDefaultMaterial(&m);
            materials.push_back(m);
        }
    }
    // Non-finite vertex positions (an OBJ coordinate past FLT_MAX parses to inf; a transform
    // can overflow too) are refused: the SAH builder's centroid bounds and bucket indices
    // are undefined on them -- the reference's build, restated exactly, did not finish on
    // such a file within a minute (a fuzzed OBJ) -- and no ray can hit such a triangle.
    for (size_t i = meshIndexBase; i < meshes.size(); ++i)
        for (const dcrt_vertex& v : meshes[i].vertices)
            if (!std::isfinite(v.position[0]) || !std::isfinite(v.position[1]) || !std::isfinite(v.position[2])) {
                SetLastError("non-finite vertex position in mesh " + std::to_string(i));
                return false;
            }
    // BLAS per new mesh (Scene.cpp:162-172)
    {
        std::vector<uint32_t> reordered;
        for (size_t i = meshIndexBase; i < meshes.size(); ++i) meshes[i].BuildBVH(&reordered);
    }
    // TLAS over all instances (Scene.cpp:174-215)
    tlas.clear();
    {
        const uint32_t instanceCount = (uint32_t)meshInstances.size();
        std::vector<bvh::Instance> blas(instanceCount);
        for (uint32_t i = 0; i < instanceCount; ++i) {
            const Mesh& mesh = meshes[meshInstances[i].meshIndex];
            if (mesh.bvhNodes.empty()) return false;
            blas[i].box = mesh.bvhNodes[0].box;
            blas[i].transform = instanceTransforms[i].To4x4();
            // a non-finite instance box (an overflowing transform: a fuzzed XML matrix entry of
            // 3e9612 never let the TLAS build finish) is refused like a non-finite vertex
            const BoundingBox world = BoxTransform(blas[i].box, blas[i].transform);
            const Float3 c = world.center, e = world.extents;
            if (!std::isfinite(c.x) || !std::isfinite(c.y) || !std::isfinite(c.z) || !std::isfinite(e.x) || !std::isfinite(e.y) ||
                !std::isfinite(e.z)) {
                SetLastError("non-finite bounds of instance " + std::to_string(i) + " (its transform)");
                return false;
            }
        }
        std::vector<uint32_t> depths(instanceCount);
        originalInstanceIndices.assign(instanceCount, 0);
        bvh::BuildResult result;
        bvh::BuildTLAS(blas.data(), instanceCount, originalInstanceIndices.data(), depths.data(), &result);
        tlas = std::move(result.nodes);
        uint32_t maxStack = 0;
        for (uint32_t i = 0; i < instanceCount; ++i) {
            const uint32_t mesh = meshInstances[originalInstanceIndices[i]].meshIndex;
            maxStack = std::max(maxStack, depths[i] + meshes[mesh].bvhMaxDepth);
        }
        bvhTraversalStackSize = maxStack;
        reorderedInstanceIndices.assign(instanceCount, 0);
        for (uint32_t r = 0; r < instanceCount; ++r) reorderedInstanceIndices[originalInstanceIndices[r]] = r;
    }
    // Mesh flags (Scene.cpp:62-90)
    meshOpaque.resize(meshes.size());
    for (size_t i = 0; i < meshes.size(); ++i) {
        bool opaque = true;
        for (uint32_t id : meshes[i].materialIds) opaque = opaque && materials[id].IsOpaque();
        meshOpaque[i] = opaque;
    }
    uint64_t totalNodes = tlas.size();
    for (const Mesh& m : meshes) totalNodes += m.bvhNodes.size();
    if (totalNodes > 2147483647ull) return false;   // Scene.cpp:266-271
    Flatten();
    hasValidScene = true;
    return true;
}

void CScene::FillMaterial(dcrt_material* out, const SMaterial& s) const
{
    // Scene.cpp:750-766
    const Float3 albedo = s.type == EMaterialType::Conductor ? s.k : s.albedo;
    out->albedo[0] = albedo.x; out->albedo[1] = albedo.y; out->albedo[2] = albedo.z;
    out->albedo_texture_index = (s.type == EMaterialType::Conductor || s.type == EMaterialType::Dielectric) ? -1 : s.albedoTextureIndex;
    out->ior[0] = s.ior.x; out->ior[1] = s.ior.y; out->ior[2] = s.ior.z;
    out->roughness = std::clamp(s.roughness, 0.0f, 1.0f);
    out->tex_tiling[0] = s.tiling.x; out->tex_tiling[1] = s.tiling.y;
    out->opacity = s.opacity;
    out->opacity_texture_index = s.opacityTextureIndex;
    uint32_t flags = (uint32_t)s.type & DCRT_MATERIAL_FLAG_TYPE_MASK;
    flags |= s.multiscattering ? DCRT_MATERIAL_FLAG_MULTISCATTERING : 0u;
    flags |= s.isTwoSided ? DCRT_MATERIAL_FLAG_IS_TWOSIDED : 0u;
    flags |= s.hasRoughnessTexture ? DCRT_MATERIAL_FLAG_ROUGHNESS_TEXTURE : 0u;
    flags |= (s.internalScatteringMode << DCRT_MATERIAL_FLAG_INTERNAL_SCATTERING_SHIFT) & DCRT_MATERIAL_FLAG_INTERNAL_SCATTERING_MASK;
    out->flags = flags;
}

static inline float AsFloat(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }

void CScene::Flatten()
{
    const uint32_t instanceCount = (uint32_t)meshInstances.size();
    // vertices (Scene.cpp:273-300)
    flatVertices_.clear();
    for (const Mesh& m : meshes) flatVertices_.insert(flatVertices_.end(), m.vertices.begin(), m.vertices.end());
    // triangles (Scene.cpp:302-335)
    flatTriangles_.clear();
    {
        uint32_t offset = 0;
        for (const Mesh& m : meshes) {
            for (uint32_t idx : m.indices) flatTriangles_.push_back(idx + offset);
            offset += (uint32_t)m.vertices.size();
        }
    }
    // BVH nodes (Scene.cpp:337-391)
    {
        uint32_t total = (uint32_t)tlas.size();
        for (const Mesh& m : meshes) total += (uint32_t)m.bvhNodes.size();
        flatNodes_.assign(total, dcrt_bvh_node{});
        std::vector<uint32_t> blasOffsets;
        uint32_t triOffset = 0, nodeOffset = (uint32_t)tlas.size();
        dcrt_bvh_node* dest = flatNodes_.data() + tlas.size();
        for (const Mesh& m : meshes) {
            bvh::PackBVH(m.bvhNodes.data(), (uint32_t)m.bvhNodes.size(), true, dest, nodeOffset, triOffset);
            dest += m.bvhNodes.size();
            blasOffsets.push_back(nodeOffset);
            triOffset += m.GetTriangleCount();
            nodeOffset += (uint32_t)m.bvhNodes.size();
        }
        std::vector<bvh::Node> t = tlas;
        for (bvh::Node& n : t) {
            if (n.primCountOrInstance > 0 || n.isLeaf) {
                const uint32_t prim = n.childOrPrimIndex;
                const uint32_t mesh = meshInstances[originalInstanceIndices[prim]].meshIndex;
                n.childOrPrimIndex = blasOffsets[mesh];
                n.primCountOrInstance = prim;
            }
        }
        bvh::PackBVH(t.data(), (uint32_t)t.size(), false, flatNodes_.data());
        tlasNodeCount_ = (uint32_t)tlas.size();
    }
    // material ids (Scene.cpp:393-421)
    flatMaterialIds_.clear();
    for (const Mesh& m : meshes) flatMaterialIds_.insert(flatMaterialIds_.end(), m.materialIds.begin(), m.materialIds.end());
    // instance transforms: forward then inverse, column-major (Scene.cpp:423-465)
    flatTransforms_.assign(instanceCount * 2, dcrt_float4x3{});
    for (uint32_t i = 0; i < instanceCount; ++i) {
        const Float4x3& T = instanceTransforms[originalInstanceIndices[i]];
        const Float4x3 I = Float4x3::From4x4(Inverse(T.To4x4()));
        for (int c = 0; c < 3; ++c)
            for (int r = 0; r < 4; ++r) {
                flatTransforms_[i].m[c * 4 + r] = T.m[r][c];
                flatTransforms_[instanceCount + i].m[c * 4 + r] = I.m[r][c];
            }
    }
    // instance light indices (Scene.cpp:467-499)
    flatLightIndices_.assign(instanceCount, DCRT_LIGHT_INDEX_INVALID);
    for (uint32_t li = 0; li < meshLights.size(); ++li)
        flatLightIndices_[reorderedInstanceIndices[meshLights[li].instanceIndex]] = li;
    // instance flags (Scene.cpp:776-807)
    flatInstanceFlags_.assign(instanceCount, 0u);
    for (uint32_t i = 0; i < instanceCount; ++i) {
        const SMeshInstance& inst = meshInstances[originalInstanceIndices[i]];
        const bool opaque = inst.materialIdOverride != kInvalidMaterialId ? materials[inst.materialIdOverride].IsOpaque()
                                                                          : (bool)meshOpaque[inst.meshIndex];
        flatInstanceFlags_[i] = opaque ? DCRT_INSTANCE_FLAG_OPAQUE : 0u;
    }
    // material overrides (Scene.cpp:522-552)
    flatOverrides_.assign(instanceCount, 0u);
    for (uint32_t i = 0; i < instanceCount; ++i) flatOverrides_[i] = meshInstances[originalInstanceIndices[i]].materialIdOverride;
    // materials (Scene.cpp:742-774)
    flatMaterials_.assign(materials.size(), dcrt_material{});
    for (size_t i = 0; i < materials.size(); ++i) FillMaterial(&flatMaterials_[i], materials[i]);
    // lights: mesh, environment, punctual (Scene.cpp:672-735)
    flatLights_.clear();
    {
        std::vector<uint32_t> triOffsets;
        uint32_t tc = 0;
        for (const Mesh& m : meshes) { triOffsets.push_back(tc); tc += m.GetTriangleCount(); }
        for (const SMeshLight& ml : meshLights) {
            dcrt_light l{};
            l.radiance[0] = ml.color.x; l.radiance[1] = ml.color.y; l.radiance[2] = ml.color.z;
            const uint32_t mesh = meshInstances[ml.instanceIndex].meshIndex;
            l.position_or_triangle_range[0] = AsFloat(triOffsets[mesh]);
            l.position_or_triangle_range[1] = AsFloat(meshes[mesh].GetTriangleCount());
            l.position_or_triangle_range[2] = AsFloat(reorderedInstanceIndices[ml.instanceIndex]);
            l.flags = DCRT_LIGHT_FLAGS_MESH_LIGHT;
            flatLights_.push_back(l);
        }
        if (hasEnvironmentLight) {
            dcrt_light l{};
            l.radiance[0] = environmentLight.color.x; l.radiance[1] = environmentLight.color.y; l.radiance[2] = environmentLight.color.z;
            l.flags = DCRT_LIGHT_FLAGS_ENVIRONMENT_LIGHT;
            flatLights_.push_back(l);
        }
        for (const SPunctualLight& pl : punctualLights) {
            dcrt_light l{};
            l.radiance[0] = pl.color.x; l.radiance[1] = pl.color.y; l.radiance[2] = pl.color.z;
            const Float3 p = pl.isDirectional ? pl.CalculateDirection() : pl.position;
            l.position_or_triangle_range[0] = p.x; l.position_or_triangle_range[1] = p.y; l.position_or_triangle_range[2] = p.z;
            l.flags = pl.isDirectional ? DCRT_LIGHT_FLAGS_DIRECTIONAL_LIGHT : DCRT_LIGHT_FLAGS_POINT_LIGHT;
            flatLights_.push_back(l);
        }
    }
    flatTextures_.clear();
    for (const CTexture& t : textures) {
        dcrt_texture d{};
        d.width = t.IsValid() ? t.width : 0;
        d.height = t.IsValid() ? t.height : 0;
        d.format = t.format;
        d.pixels = t.IsValid() ? t.pixels.data() : nullptr;
        flatTextures_.push_back(d);
    }
}

dcrt_flat_scene CScene::GetFlat() const
{
    dcrt_flat_scene f{};
    f.vertices = flatVertices_.data(); f.vertex_count = (uint32_t)flatVertices_.size();
    f.triangles = flatTriangles_.data(); f.triangle_count = (uint32_t)flatTriangles_.size() / 3;
    f.bvh_nodes = flatNodes_.data(); f.bvh_node_count = (uint32_t)flatNodes_.size();
    f.tlas_node_count = tlasNodeCount_;
    f.material_ids = flatMaterialIds_.data();
    f.instance_transforms = flatTransforms_.data(); f.instance_count = (uint32_t)meshInstances.size();
    f.instance_light_indices = flatLightIndices_.data();
    f.instance_flags = flatInstanceFlags_.data();
    f.instance_material_overrides = flatOverrides_.data();
    f.materials = flatMaterials_.data(); f.material_count = (uint32_t)flatMaterials_.size();
    f.lights = flatLights_.data(); f.light_count = (uint32_t)flatLights_.size();
    f.environment_light_index = hasEnvironmentLight ? (uint32_t)meshLights.size() : DCRT_LIGHT_INDEX_INVALID;
    f.textures = flatTextures_.data(); f.texture_count = (uint32_t)flatTextures_.size();
    f.env_cube_rgb = (hasEnvironmentLight && environmentLight.cubeSize) ? environmentLight.cubeRGB.data() : nullptr;
    f.env_cube_size = (hasEnvironmentLight && environmentLight.cubeSize) ? environmentLight.cubeSize : 0;
    f.bvh_traversal_stack_size = bvhTraversalStackSize;
    return f;
}

dcrt_frame_params CScene::GetFrameParams(uint32_t frameSeed) const
{
    dcrt_frame_params p{};
    const Float4x4 cam = camera.GetTransformMatrix();
    for (int r = 0; r < 4; ++r) for (int c = 0; c < 4; ++c) p.camera_transform[r * 4 + c] = cam.m[r][c];
    p.resolution[0] = resolutionWidth;
    p.resolution[1] = resolutionHeight;
    p.film_size[0] = filmSize.x;
    p.film_size[1] = filmSize.y;
    p.aperture_radius = CalculateApertureDiameter() * 0.5f;
    p.focal_distance = focalDistance;
    p.film_distance = CalculateFilmDistance();
    p.blade_count = apertureBladeCount;
    const float halfBladeAngle = 3.141592654f / (float)apertureBladeCount;   // DirectX::XM_PI
    p.blade_vertex_pos[0] = std::cos(halfBladeAngle) * p.aperture_radius;
    p.blade_vertex_pos[1] = std::sin(halfBladeAngle) * p.aperture_radius;
    p.aperture_base_angle = apertureRotation;
    p.frame_seed = frameSeed;
    p.max_bounce_count = maxBounceCount;
    p.light_count = GetLightCount();
    p.environment_light_index = hasEnvironmentLight ? (uint32_t)meshLights.size() : DCRT_LIGHT_INDEX_INVALID;
    p.features = features;
    return p;
}

dcrt_filter_params CScene::GetFilterParams() const
{
    dcrt_filter_params f{};
    f.filter = (uint32_t)filter;
    f.radius = filterRadius;
    f.gaussian_alpha = gaussianFilterAlpha;
    f.mitchell_b = mitchellB;
    f.mitchell_c = mitchellC;
    f.lanczos_tau = lanczosSincTau;
    return f;
}

// ---------------------------------------------------------------- OBJ scene (WavefrontOBJLoading.cpp:409-465)
bool CScene::LoadFromWavefrontOBJFile(const std::string& path)
{
    ObjData data;
    std::string err;
    if (!ParseObjFile(path, &data, &err)) {
        std::fprintf(stderr, "dcrt: OBJ load failed: %s\n", err.c_str());
        return false;
    }
    SMeshProcessingParams params;
    params.applyTransform = true;
    params.transform = Float4x4::Identity();
    params.transform.m[0][0] = -1.0f;      // RH -> LH
    params.changeWindingOrder = true;
    params.flipTexcoordV = true;
    for (size_t s = 0; s < data.shapes.size(); ++s) {
        meshes.emplace_back();
        params.materialIndexBase = (uint32_t)materials.size();
        Mesh& mesh = meshes.back();
        if (!CreateMeshFromObjData(data, &data.shapes[s], 1, params, &mesh)) return false;
        mesh.name = data.shapes[s].name;
        SMeshInstance inst;
        inst.name = mesh.name;
        inst.meshIndex = (uint32_t)meshes.size() - 1;
        inst.materialIdOverride = kInvalidMaterialId;
        meshInstances.push_back(inst);
        instanceTransforms.push_back(Float4x3::Identity());
    }
    std::vector<std::string> textureNames;
    TranslateObjMaterials(data, (int32_t)textures.size(), &materials, &textureNames);
    const std::string dir = path.find_last_of('/') == std::string::npos ? std::string(".") : path.substr(0, path.find_last_of('/'));
    for (const std::string& name : textureNames) {
        CTexture t;
        t.name = name;
        const std::string full = (!name.empty() && name[0] == '/') ? name : dir + "/" + name;
        if (!LoadTextureFile(full, &t)) std::fprintf(stderr, "dcrt: loading texture \"%s\" failed\n", full.c_str());
        textures.push_back(std::move(t));
    }
    return true;
}

bool CScene::LoadFromXMLFile(const std::string& path) { return LoadMitsubaXML(this, path); }

}  // namespace dcrt
