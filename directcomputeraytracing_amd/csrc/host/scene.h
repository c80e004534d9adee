// scene.h -- CScene / Mesh / Camera host model (Source/Scene.h, Mesh.h,
// Camera.h, Material.h) and its flattening into the Appendix-B wire format
// that the MI355X tracer uploads (Scene.cpp:273-608, 672-807).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

#include "../../../include/dcrt.h"
#include "bvh_accel.h"
#include "xmath.h"

namespace dcrt {

constexpr uint32_t kInvalidMaterialId = 0xFFFFFFFFu;   // Constants.h:8
constexpr float kMaxMaterialIor = 3.0f;                // Constants.h:3

enum class EMaterialType : uint32_t { Diffuse = 0, Plastic = 1, Conductor = 2, Dielectric = 3, ThinDielectric = 4 };
enum class ECameraType : uint32_t { PinHole = 0, ThinLens = 1 };
enum class EFilter : uint32_t { Box = 0, Triangle = 1, Gaussian = 2, Mitchell = 3, LanczosSinc = 4 };

// Material.h:14-30
struct SMaterial {
    Float3 albedo{ 1.0f, 0.0f, 1.0f };
    float roughness = 1.0f;
    Float3 ior{ 1.0f, 1.0f, 1.0f };
    float opacity = 1.0f;
    Float3 k{ 1.0f, 1.0f, 1.0f };
    Float2 tiling{ 1.0f, 1.0f };
    std::string name;
    EMaterialType type = EMaterialType::Diffuse;
    int32_t albedoTextureIndex = -1;
    int32_t opacityTextureIndex = -1;
    uint32_t internalScatteringMode = DCRT_INTERNAL_SCATTERING_MULTIPLE;
    bool multiscattering = false;
    bool isTwoSided = false;
    bool hasRoughnessTexture = false;
    bool IsOpaque() const { return opacity == 1.0f && opacityTextureIndex == -1; }   // Scene.cpp:57-60
};
void GetDefaultMaterial(SMaterial* material);   // Scene.cpp:39-55

// Mesh.h:19-67
struct Mesh {
    std::string name;
    std::vector<dcrt_vertex> vertices;
    std::vector<uint32_t> indices;
    std::vector<bvh::Node> bvhNodes;
    uint32_t bvhMaxDepth = 0;
    uint32_t bvhMaxStackSize = 0;
    std::vector<uint32_t> materialIds;
    std::vector<uint32_t> bvhTriangleOrder;   // BVH position -> load-order triangle (BuildBLAS output)

    uint32_t GetTriangleCount() const { return (uint32_t)indices.size() / 3; }
    void BuildBVH(std::vector<uint32_t>* reorderedTriangleIndices);   // Mesh.cpp:59-79
    bool GenerateRectangle(uint32_t materialId, bool applyTransform, const Float4x4& transform);   // Mesh.cpp:7-57
};

struct SMeshInstance { std::string name; uint32_t meshIndex = 0; uint32_t materialIdOverride = kInvalidMaterialId; };
struct SPunctualLight {
    Float3 position, eulerAngles, color;
    bool isDirectional = false;
    Float3 CalculateDirection() const;                       // Scene.cpp:946-955
    void SetEulerAnglesFromDirection(const Float3& dir);     // Scene.cpp:913-944
};
struct SMeshLight { uint32_t instanceIndex = 0; Float3 color; };
struct SEnvironmentLight { Float3 color{ 1.0f, 1.0f, 1.0f }; std::vector<float> cubeRGB; uint32_t cubeSize = 0; };
struct CTexture { std::string name; uint32_t width = 0, height = 0, format = DCRT_TEXTURE_FORMAT_RGBA8_SRGB; std::vector<uint8_t> pixels; bool IsValid() const { return width && height && !pixels.empty(); } };

// Camera.cpp:6-96 (UI motion is out of scope)
struct Camera {
    Float3 position{ 0.0f, 1.0f, 0.0f };
    Float3 eulerAngles{ 0.0f, 0.0f, 0.0f };
    Float4x4 GetTransformMatrix() const;
};

struct SMeshProcessingParams {   // Mesh.h:9-17
    Float4x4 transform = Float4x4::Identity();
    uint32_t materialIndexBase = 0;
    uint32_t textureIndexBase = 0;
    bool applyTransform = false;
    bool changeWindingOrder = false;
    bool flipTexcoordV = false;
};

class CScene {
public:
    bool LoadFromFile(const std::string& path);   // Scene.cpp:103-624
    void Reset(uint32_t resolutionWidth, uint32_t resolutionHeight);   // Scene.cpp:626-660
    uint32_t GetLightCount() const { return (uint32_t)(meshLights.size() + punctualLights.size() + (hasEnvironmentLight ? 1 : 0)); }
    float CalculateFilmDistance() const;           // Scene.cpp:837-842
    float CalculateApertureDiameter() const;       // Scene.cpp:844-847

    // Rebuilds the flat arrays (GPU buffer contents) and returns views of them.
    void Flatten();
    dcrt_flat_scene GetFlat() const;
    dcrt_frame_params GetFrameParams(uint32_t frameSeed) const;   // WavefrontPathTracer.cpp:372-428
    dcrt_filter_params GetFilterParams() const;

    // ---- public state (Scene.h:118-160) ----
    uint32_t resolutionWidth = 1920, resolutionHeight = 1080;
    Float2 filmSize{ 0.05333f, 0.03f };
    ECameraType cameraType = ECameraType::ThinLens;
    float fovX = 1.221730f;
    float focalLength = 0.05f;
    float focalDistance = 2.0f;
    float relativeAperture = 8.0f;
    uint32_t apertureBladeCount = 7;
    float apertureRotation = 0.0f;
    float shutterTime = 1.0f;
    float iso = 100.0f;
    uint32_t maxBounceCount = 2;
    float filterRadius = 1.0f;
    EFilter filter = EFilter::Box;
    float gaussianFilterAlpha = 1.5f;
    float mitchellB = 1.0f / 3.0f;
    float mitchellC = 1.0f / 3.0f;
    uint32_t lanczosSincTau = 3;
    uint32_t features = DCRT_FEATURE_DEFAULT;

    Camera camera;
    bool hasEnvironmentLight = false;
    SEnvironmentLight environmentLight;
    std::vector<SPunctualLight> punctualLights;
    std::vector<SMeshLight> meshLights;
    std::vector<SMaterial> materials;
    std::vector<Mesh> meshes;
    std::vector<bool> meshOpaque;                   // SMeshFlags::m_Opaque
    std::vector<SMeshInstance> meshInstances;
    std::vector<bvh::Node> tlas;
    std::vector<uint32_t> originalInstanceIndices;  // reordered -> original
    std::vector<uint32_t> reorderedInstanceIndices; // original -> reordered
    std::vector<Float4x3> instanceTransforms;
    std::vector<CTexture> textures;
    uint32_t bvhTraversalStackSize = 0;
    bool hasValidScene = false;

private:
    bool LoadFromWavefrontOBJFile(const std::string& path);
    bool LoadFromXMLFile(const std::string& path);
    void FillMaterial(dcrt_material* out, const SMaterial& in) const;

    // flat storage (the buffers of Scene.cpp:273-608)
    std::vector<dcrt_vertex> flatVertices_;
    std::vector<uint32_t> flatTriangles_;
    std::vector<dcrt_bvh_node> flatNodes_;
    std::vector<uint32_t> flatMaterialIds_;
    std::vector<dcrt_float4x3> flatTransforms_;
    std::vector<uint32_t> flatLightIndices_;
    std::vector<uint32_t> flatInstanceFlags_;
    std::vector<uint32_t> flatOverrides_;
    std::vector<dcrt_material> flatMaterials_;
    std::vector<dcrt_light> flatLights_;
    std::vector<dcrt_texture> flatTextures_;
    uint32_t tlasNodeCount_ = 0;
    friend bool LoadMitsubaXML(CScene* scene, const std::string& path);
// The element / attribute tree the XML loader parsed (tests: compared with rapidxml's)
bool DumpXmlTree(const std::string& path, std::string* out);
};

// OBJ parsing (the tinyobjloader subset WavefrontOBJLoading.cpp relies on).
struct ObjIndex { int v = -1, vn = -1, vt = -1; };
struct ObjShape { std::string name; std::vector<ObjIndex> indices; std::vector<int> materialIds; };
struct ObjMaterial {
    std::string name;
    float diffuse[3] = { 0.0f, 0.0f, 0.0f };
    float ior = 1.0f, dissolve = 1.0f, roughness = 0.0f;
    std::string diffuseTexname, alphaTexname;
};
struct ObjData {
    std::vector<float> positions, normals, texcoords;
    std::vector<ObjShape> shapes;
    std::vector<ObjMaterial> materials;
};
bool ParseObjFile(const std::string& path, ObjData* out, std::string* err);
bool CreateMeshFromObjData(const ObjData& data, const ObjShape* shapes, uint32_t shapeCount,
                           const SMeshProcessingParams& params, Mesh* outMesh);
void TranslateObjMaterials(const ObjData& data, int32_t textureIndexBase, std::vector<SMaterial>* out,
                           std::vector<std::string>* textureNames);
bool LoadMitsubaXML(CScene* scene, const std::string& path);
// The element / attribute tree the XML loader parsed (tests: compared with rapidxml's)
bool DumpXmlTree(const std::string& path, std::string* out);
bool LoadTextureFile(const std::string& path, CTexture* out);
// MikkTSpace genTangSpaceDefault over a triangle list given per corner (3 per triangle;
// texcoords carry z = 1); false for an empty list (tangent_space.cpp).
bool GenerateMikkTangents(const std::vector<Float3>& positions, const std::vector<Float3>& normals,
                          const std::vector<Float3>& texcoords, std::vector<Float3>* out);

}  // namespace dcrt
