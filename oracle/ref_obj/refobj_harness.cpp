// TEST INFRASTRUCTURE -- never part of the product, never measured.
//
// The reference's OBJ load flow (Source/WavefrontOBJLoading.cpp:155-263 mesh creation,
// :374-407 Mesh::LoadFromWavefrontOBJFile, :409-465 CScene::LoadFromWavefrontOBJFile)
// restated around the UNMODIFIED third-party libraries it uses, compiled from
// /root/reference by oracle/ref_obj/Makefile:
//   * tinyobjloader (tinyobjloader/tiny_obj_loader.h, LoadObj with triangulation)
//   * MikkTSpace (MikkTSpace/mikktspace.c, genTangSpaceDefault)
// DirectXMath is not available here; the RH->LH transform uses the XMVector3Transform /
// XMVector3TransformNormal SSE operation order with the exact inverse of diag(-1,1,1,1)
// (+0 off the diagonal; the sign of those zeros in XMMatrixInverse is parity unpinned).
// tests/test_obj_pin.py compares the product's dcrt_obj_load with this bit for bit.
#define TINYOBJLOADER_IMPLEMENTATION
#include "tinyobjloader/tiny_obj_loader.h"
#include "MikkTSpace/mikktspace.h"

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <unordered_map>
#include <vector>

namespace {

struct RefVertex { float pos[3], nrm[3], tan[3], uv[2]; };
struct RefMesh { std::vector<RefVertex> vertices; std::vector<uint32_t> indices, materialIds; };
struct RefMaterial { float albedo[3], ior, roughness, opacity; int32_t albedoTex, opacityTex; };
struct RefLoad { std::vector<RefMesh> meshes; std::vector<RefMaterial> materials; };

struct MikkView {
    const tinyobj::attrib_t* attrib;
    const tinyobj::mesh_t* mesh;
    std::vector<float>* tangents;   // 3 per corner
    bool flipV;
};

MikkView* View(const SMikkTSpaceContext* c) { return static_cast<MikkView*>(c->m_pUserData); }
int NumFaces(const SMikkTSpaceContext* c) { return (int)View(c)->mesh->num_face_vertices.size(); }
int NumVerts(const SMikkTSpaceContext*, const int) { return 3; }
void Position(const SMikkTSpaceContext* c, float out[], const int f, const int v)
{
    const tinyobj::index_t i = View(c)->mesh->indices[f * 3 + v];
    for (int k = 0; k < 3; ++k) out[k] = View(c)->attrib->vertices[i.vertex_index * 3 + k];
}
void Normal(const SMikkTSpaceContext* c, float out[], const int f, const int v)
{
    const tinyobj::index_t i = View(c)->mesh->indices[f * 3 + v];
    for (int k = 0; k < 3; ++k) out[k] = View(c)->attrib->normals[i.normal_index * 3 + k];
}
void TexCoord(const SMikkTSpaceContext* c, float out[], const int f, const int v)
{
    const tinyobj::index_t i = View(c)->mesh->indices[f * 3 + v];
    if (i.texcoord_index == -1) { out[0] = out[1] = 0.0f; return; }
    out[0] = View(c)->attrib->texcoords[i.texcoord_index * 2];
    out[1] = View(c)->attrib->texcoords[i.texcoord_index * 2 + 1];
    if (View(c)->flipV) out[1] = 1.0f - out[1];
}
void SetBasic(const SMikkTSpaceContext* c, const float t[], const float, const int f, const int v)
{
    float* d = &(*View(c)->tangents)[(size_t)(f * 3 + v) * 3];
    d[0] = t[0]; d[1] = t[1]; d[2] = t[2];
}

struct Key {
    int v, vn, vt;
    float t[3];
    bool operator==(const Key& o) const
    {
        return v == o.v && vn == o.vn && vt == o.vt && t[0] == o.t[0] && t[1] == o.t[1] && t[2] == o.t[2];
    }
};
struct KeyHash {
    size_t operator()(const Key& k) const
    {
        auto f = [](float x) { return x == 0.0f ? (size_t)0 : std::hash<float>()(x); };
        return std::hash<int>()(k.v) * 31u ^ std::hash<int>()(k.vn) * 131u ^ std::hash<int>()(k.vt) * 1031u ^
               f(k.t[0]) * 7u ^ f(k.t[1]) * 17u ^ f(k.t[2]) * 29u;
    }
};

// XMVector3Transform / XMVector3TransformNormal with M = N = diag(-1, 1, 1, 1)
const float kM[4][3] = { { -1.0f, 0.0f, 0.0f }, { 0.0f, 1.0f, 0.0f }, { 0.0f, 0.0f, 1.0f }, { 0.0f, 0.0f, 0.0f } };
void XformPoint(float p[3])
{
    float r[3];
    for (int c = 0; c < 3; ++c) {
        float t = p[2] * kM[2][c] + kM[3][c];
        t = p[1] * kM[1][c] + t;
        r[c] = p[0] * kM[0][c] + t;
    }
    std::memcpy(p, r, sizeof(r));
}
void XformNormal(float n[3])
{
    float r[3];
    for (int c = 0; c < 3; ++c) {
        float t = n[2] * kM[2][c];
        t = n[1] * kM[1][c] + t;
        r[c] = n[0] * kM[0][c] + t;
    }
    std::memcpy(n, r, sizeof(r));
}

// CreateMeshFromWavefrontOBJData (WavefrontOBJLoading.cpp:155-263)
bool CreateMesh(const tinyobj::attrib_t& attrib, const tinyobj::shape_t* shapes, size_t count, bool transform,
                uint32_t materialBase, RefMesh* out)
{
    if (attrib.normals.size() / 3 == 0) return false;
    SMikkTSpaceInterface iface;
    std::memset(&iface, 0, sizeof(iface));
    iface.m_getNumFaces = NumFaces;
    iface.m_getNumVerticesOfFace = NumVerts;
    iface.m_getPosition = Position;
    iface.m_getNormal = Normal;
    iface.m_getTexCoord = TexCoord;
    iface.m_setTSpaceBasic = SetBasic;
    SMikkTSpaceContext ctx;
    ctx.m_pInterface = &iface;
    static const int kWinding[3] = { 0, 2, 1 };   // m_ChangeWindingOrder is always set by the callers
    std::unordered_map<Key, uint32_t, KeyHash> seen;
    std::vector<float> tangents;
    for (size_t s = 0; s < count; ++s) {
        const tinyobj::mesh_t& mesh = shapes[s].mesh;
        tangents.assign(mesh.num_face_vertices.size() * 9, 0.0f);
        MikkView view{ &attrib, &mesh, &tangents, true };
        ctx.m_pUserData = &view;
        if (!genTangSpaceDefault(&ctx)) continue;
        for (size_t f = 0; f < mesh.num_face_vertices.size(); ++f) {
            const int mat = mesh.material_ids[f];
            out->materialIds.push_back(mat != -1 ? materialBase + (uint32_t)mat : 0xFFFFFFFFu);
            for (int k = 0; k < 3; ++k) {
                const size_t corner = f * 3 + kWinding[k];
                const tinyobj::index_t idx = mesh.indices[corner];
                if (idx.vertex_index == -1 || idx.normal_index == -1) return false;
                Key key{ idx.vertex_index, idx.normal_index, idx.texcoord_index,
                         { tangents[corner * 3], tangents[corner * 3 + 1], tangents[corner * 3 + 2] } };
                auto it = seen.find(key);
                uint32_t vi;
                if (it != seen.end()) {
                    vi = it->second;
                } else {
                    vi = (uint32_t)out->vertices.size();
                    RefVertex v;
                    for (int c = 0; c < 3; ++c) {
                        v.pos[c] = attrib.vertices[idx.vertex_index * 3 + c];
                        v.nrm[c] = attrib.normals[idx.normal_index * 3 + c];
                        v.tan[c] = key.t[c];
                    }
                    if (idx.texcoord_index != -1) {
                        v.uv[0] = attrib.texcoords[idx.texcoord_index * 2];
                        v.uv[1] = attrib.texcoords[idx.texcoord_index * 2 + 1];
                    } else {
                        v.uv[0] = v.uv[1] = 0.0f;
                    }
                    v.uv[1] = 1.0f - v.uv[1];
                    if (transform) { XformPoint(v.pos); XformNormal(v.nrm); XformNormal(v.tan); }
                    out->vertices.push_back(v);
                    seen.insert({ key, vi });
                }
                out->indices.push_back(vi);
            }
        }
    }
    return true;
}

// SMaterialTranslationContext::TranslateMaterials (WavefrontOBJLoading.cpp:285-338)
void TranslateMaterials(const std::vector<tinyobj::material_t>& src, std::vector<RefMaterial>* out)
{
    std::unordered_map<std::string, int32_t> tex;
    auto getTex = [&](const std::string& n) {
        auto it = tex.find(n);
        if (it != tex.end()) return it->second;
        const int32_t i = (int32_t)tex.size();
        tex.insert({ n, i });
        return i;
    };
    for (const tinyobj::material_t& m : src) {
        RefMaterial r;
        for (int c = 0; c < 3; ++c) r.albedo[c] = m.diffuse[c];
        r.roughness = m.roughness;
        r.ior = std::clamp(m.ior, 1.0f, 3.0f);   // MAX_MATERIAL_IOR (Constants.h)
        r.opacity = m.dissolve;
        r.albedoTex = m.diffuse_texname.length() > 0 ? getTex(m.diffuse_texname) : -1;
        r.opacityTex = m.alpha_texname.length() > 0 ? getTex(m.alpha_texname) : -1;
        out->push_back(r);
    }
}

}  // namespace

extern "C" {

// scene_layout 1: CScene::LoadFromWavefrontOBJFile (a mesh per shape, RH->LH);
//              0: Mesh::LoadFromWavefrontOBJFile as SceneXMLLoading.cpp:1334-1341 calls it
int refobj_load(const char* path, int sceneLayout, uint32_t materialBase, void** out)
{
    tinyobj::attrib_t attrib;
    std::vector<tinyobj::shape_t> shapes;
    std::vector<tinyobj::material_t> materials;
    std::string warn, err;
    const std::string file(path);
    const size_t slash = file.find_last_of('/');
    const std::string dir = slash == std::string::npos ? std::string() : (slash == 0 ? std::string("/") : file.substr(0, slash));
    if (!tinyobj::LoadObj(&attrib, &shapes, &materials, &warn, &err, path, dir.c_str())) return -1;
    RefLoad* r = new RefLoad();
    if (sceneLayout) {
        for (size_t s = 0; s < shapes.size(); ++s) {
            r->meshes.emplace_back();
            if (!CreateMesh(attrib, &shapes[s], 1, true, materialBase, &r->meshes.back())) { delete r; return -2; }
        }
    } else {
        r->meshes.emplace_back();
        if (!CreateMesh(attrib, shapes.data(), shapes.size(), false, materialBase, &r->meshes.back())) { delete r; return -2; }
    }
    TranslateMaterials(materials, &r->materials);
    *out = r;
    return 0;
}

int refobj_mesh_count(void* h) { return (int)static_cast<RefLoad*>(h)->meshes.size(); }

int refobj_get_mesh(void* h, int i, const float** vertices, uint32_t* vertexCount, const uint32_t** indices,
                    const uint32_t** materialIds, uint32_t* triangleCount)
{
    const RefMesh& m = static_cast<RefLoad*>(h)->meshes.at((size_t)i);
    *vertices = m.vertices.empty() ? nullptr : m.vertices[0].pos;
    *vertexCount = (uint32_t)m.vertices.size();
    *indices = m.indices.data();
    *materialIds = m.materialIds.data();
    *triangleCount = (uint32_t)m.materialIds.size();
    return 0;
}

int refobj_material_count(void* h) { return (int)static_cast<RefLoad*>(h)->materials.size(); }

int refobj_get_material(void* h, int i, float* values6, int32_t* textures2)
{
    const RefMaterial& m = static_cast<RefLoad*>(h)->materials.at((size_t)i);
    values6[0] = m.albedo[0]; values6[1] = m.albedo[1]; values6[2] = m.albedo[2];
    values6[3] = m.ior; values6[4] = m.roughness; values6[5] = m.opacity;
    textures2[0] = m.albedoTex; textures2[1] = m.opacityTex;
    return 0;
}

void refobj_free(void* h) { delete static_cast<RefLoad*>(h); }

// MikkTSpace alone over a triangle soup (3 corners per triangle), for the tangent unit tests
int refobj_mikk(const float* pos, const float* nrm, const float* uv, int triangles, float* outTangents)
{
    struct Soup { const float *p, *n, *t; float* out; int tris; };
    Soup soup{ pos, nrm, uv, outTangents, triangles };
    SMikkTSpaceInterface iface;
    std::memset(&iface, 0, sizeof(iface));
    iface.m_getNumFaces = [](const SMikkTSpaceContext* c) { return static_cast<Soup*>(c->m_pUserData)->tris; };
    iface.m_getNumVerticesOfFace = [](const SMikkTSpaceContext*, const int) { return 3; };
    iface.m_getPosition = [](const SMikkTSpaceContext* c, float o[], const int f, const int v) {
        std::memcpy(o, static_cast<Soup*>(c->m_pUserData)->p + (f * 3 + v) * 3, 12);
    };
    iface.m_getNormal = [](const SMikkTSpaceContext* c, float o[], const int f, const int v) {
        std::memcpy(o, static_cast<Soup*>(c->m_pUserData)->n + (f * 3 + v) * 3, 12);
    };
    iface.m_getTexCoord = [](const SMikkTSpaceContext* c, float o[], const int f, const int v) {
        std::memcpy(o, static_cast<Soup*>(c->m_pUserData)->t + (f * 3 + v) * 2, 8);
    };
    iface.m_setTSpaceBasic = [](const SMikkTSpaceContext* c, const float t[], const float, const int f, const int v) {
        std::memcpy(static_cast<Soup*>(c->m_pUserData)->out + (f * 3 + v) * 3, t, 12);
    };
    SMikkTSpaceContext ctx;
    ctx.m_pInterface = &iface;
    ctx.m_pUserData = &soup;
    return genTangSpaceDefault(&ctx) ? 0 : -1;
}

}  // extern "C"
