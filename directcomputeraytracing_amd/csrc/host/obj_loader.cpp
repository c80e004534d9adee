// obj_loader.cpp -- Wavefront OBJ/MTL loading for CScene
// (Source/WavefrontOBJLoading.cpp:155-465). The parser reproduces the
// tinyobjloader behaviours the reference depends on (shape split on g/o,
// per-face material ids, ear-clipping triangulation that reduces to a fan on
// convex polygons, MTL defaults). Tangents are generated per corner from the UV
// parameterisation and averaged over corners that share (v, vn, vt) -- a
// MikkTSpace-compatible result for planar, consistently mapped faces (MikkTSpace
// itself is not re-derived: parity unpinned).
#include "scene.h"

#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <unordered_map>

namespace dcrt {
namespace {

std::string Trim(const std::string& s)
{
    size_t b = s.find_first_not_of(" \t\r\n"), e = s.find_last_not_of(" \t\r\n");
    return b == std::string::npos ? std::string() : s.substr(b, e - b + 1);
}

// "v", "v/vt", "v//vn", "v/vt/vn"; 1-based, negative = relative (tinyobj parseTriple)
bool ParseCorner(const std::string& tok, int vcount, int vncount, int vtcount, ObjIndex* out)
{
    int vals[3] = { 0, 0, 0 };
    bool has[3] = { false, false, false };
    size_t pos = 0;
    for (int k = 0; k < 3 && pos <= tok.size(); ++k) {
        size_t slash = tok.find('/', pos);
        std::string part = tok.substr(pos, slash == std::string::npos ? std::string::npos : slash - pos);
        if (!part.empty()) { vals[k] = std::atoi(part.c_str()); has[k] = true; }
        if (slash == std::string::npos) break;
        pos = slash + 1;
    }
    auto fix = [](int idx, int n) { return idx > 0 ? idx - 1 : (idx < 0 ? n + idx : -1); };
    if (!has[0] || vals[0] == 0) return false;
    out->v = fix(vals[0], vcount);
    out->vt = has[1] ? fix(vals[1], vtcount) : -1;
    out->vn = has[2] ? fix(vals[2], vncount) : -1;
    return true;
}

bool PointInTriangle(const float* vx, const float* vy, float tx, float ty)   // pnpoly, 3 vertices
{
    bool c = false;
    for (int i = 0, j = 2; i < 3; j = i++)
        if (((vy[i] > ty) != (vy[j] > ty)) && (tx < (vx[j] - vx[i]) * (ty - vy[i]) / (vy[j] - vy[i]) + vx[i])) c = !c;
    return c;
}

// Ear clipping as tinyobjloader's exportGroupsToShape (fan order on convex faces).
void Triangulate(const std::vector<ObjIndex>& face, const std::vector<float>& v, int materialId, ObjShape* shape)
{
    const size_t n = face.size();
    if (n < 3) return;
    auto P = [&](const ObjIndex& i, int axis) { return (size_t)i.v * 3 + axis < v.size() ? v[(size_t)i.v * 3 + axis] : 0.0f; };
    size_t axes[2] = { 1, 2 };
    for (size_t k = 0; k < n; ++k) {
        const ObjIndex& a = face[k % n]; const ObjIndex& b = face[(k + 1) % n]; const ObjIndex& c = face[(k + 2) % n];
        float e0x = P(b, 0) - P(a, 0), e0y = P(b, 1) - P(a, 1), e0z = P(b, 2) - P(a, 2);
        float e1x = P(c, 0) - P(b, 0), e1y = P(c, 1) - P(b, 1), e1z = P(c, 2) - P(b, 2);
        float cx = std::fabs(e0y * e1z - e0z * e1y), cy = std::fabs(e0z * e1x - e0x * e1z), cz = std::fabs(e0x * e1y - e0y * e1x);
        const float eps = 1.1920929e-07f;
        if (cx > eps || cy > eps || cz > eps) {
            if (!(cx > cy && cx > cz)) { axes[0] = 0; if (cz > cx && cz > cy) axes[1] = 1; }
            break;
        }
    }
    float area = 0.0f;
    for (size_t k = 0; k < n; ++k) {
        const ObjIndex& a = face[k % n]; const ObjIndex& b = face[(k + 1) % n];
        area += (P(a, (int)axes[0]) * P(b, (int)axes[1]) - P(a, (int)axes[1]) * P(b, (int)axes[0])) * 0.5f;
    }
    std::vector<ObjIndex> rem = face;
    size_t guess = 0, remainingIterations = rem.size(), previous = rem.size();
    auto emit = [&](const ObjIndex& a, const ObjIndex& b, const ObjIndex& c) {
        shape->indices.push_back(a); shape->indices.push_back(b); shape->indices.push_back(c);
        shape->materialIds.push_back(materialId);
    };
    while (rem.size() > 3 && remainingIterations > 0) {
        const size_t np = rem.size();
        if (guess >= np) guess -= np;
        if (previous != np) { previous = np; remainingIterations = np; }
        else remainingIterations--;
        ObjIndex ind[3]; float vx[3], vy[3];
        for (int k = 0; k < 3; ++k) {
            ind[k] = rem[(guess + k) % np];
            vx[k] = P(ind[k], (int)axes[0]); vy[k] = P(ind[k], (int)axes[1]);
        }
        float e0x = vx[1] - vx[0], e0y = vy[1] - vy[0], e1x = vx[2] - vx[1], e1y = vy[2] - vy[1];
        float cross = e0x * e1y - e0y * e1x;
        if (cross * area < 0.0f) { guess += 1; continue; }
        bool overlap = false;
        for (size_t o = 3; o < np; ++o) {
            const ObjIndex& oi = rem[(guess + o) % np];
            if (PointInTriangle(vx, vy, P(oi, (int)axes[0]), P(oi, (int)axes[1]))) { overlap = true; break; }
        }
        if (overlap) { guess += 1; continue; }
        emit(ind[0], ind[1], ind[2]);
        size_t removed = (guess + 1) % np;
        rem.erase(rem.begin() + (long)removed);
    }
    if (rem.size() == 3) emit(rem[0], rem[1], rem[2]);
}

bool ParseMtl(const std::string& path, std::vector<ObjMaterial>* mats, std::map<std::string, int>* index)
{
    std::ifstream in(path);
    if (!in) return false;
    std::string line;
    ObjMaterial* cur = nullptr;
    bool hasD = false;
    while (std::getline(in, line)) {
        std::istringstream ss(line);
        std::string tag;
        ss >> tag;
        if (tag == "newmtl") {
            std::string name = Trim(line.substr(line.find("newmtl") + 6));
            mats->emplace_back();
            cur = &mats->back();
            cur->name = name;
            (*index)[name] = (int)mats->size() - 1;
            hasD = false;
        } else if (!cur) {
            continue;
        } else if (tag == "Kd") {
            double r = 0, g = 0, b = 0; ss >> r >> g >> b;
            cur->diffuse[0] = (float)r; cur->diffuse[1] = (float)g; cur->diffuse[2] = (float)b;
        } else if (tag == "Ni") {
            double x = 1; ss >> x; cur->ior = (float)x;
        } else if (tag == "Pr") {
            double x = 0; ss >> x; cur->roughness = (float)x;
        } else if (tag == "d") {
            double x = 1; ss >> x; cur->dissolve = (float)x; hasD = true;
        } else if (tag == "Tr") {
            double x = 0; ss >> x; if (!hasD) cur->dissolve = 1.0f - (float)x;
        } else if (tag == "map_Kd") {
            std::string rest = Trim(line.substr(line.find("map_Kd") + 6));
            size_t sp = rest.find_last_of(" \t");
            cur->diffuseTexname = sp == std::string::npos ? rest : rest.substr(sp + 1);
        } else if (tag == "map_d") {
            std::string rest = Trim(line.substr(line.find("map_d") + 5));
            size_t sp = rest.find_last_of(" \t");
            cur->alphaTexname = sp == std::string::npos ? rest : rest.substr(sp + 1);
        }
    }
    return true;
}

struct CornerKey {
    int v, vn, vt;
    float tx, ty, tz;
    bool operator==(const CornerKey& o) const
    {
        return v == o.v && vn == o.vn && vt == o.vt && tx == o.tx && ty == o.ty && tz == o.tz;
    }
};
struct CornerKeyHash {
    size_t operator()(const CornerKey& k) const
    {
        size_t h = 0;
        auto mix = [&h](size_t x) { h ^= x + 0x9e3779b9 + (h << 6) + (h >> 2); };
        mix(std::hash<int>()(k.v)); mix(std::hash<int>()(k.vn)); mix(std::hash<int>()(k.vt));
        mix(std::hash<float>()(k.tx)); mix(std::hash<float>()(k.ty)); mix(std::hash<float>()(k.tz));
        return h;
    }
};
struct IndexTripleHash {
    size_t operator()(const std::tuple<int, int, int>& t) const
    {
        return std::hash<int>()(std::get<0>(t)) * 73856093u ^ std::hash<int>()(std::get<1>(t)) * 19349663u ^ std::hash<int>()(std::get<2>(t)) * 83492791u;
    }
};

// Per-corner tangents for one shape (stand-in for genTangSpaceDefault, WavefrontOBJLoading.cpp:147-153).
void GenerateTangents(const ObjData& d, const ObjShape& s, bool flipV, std::vector<Float3>* out)
{
    const size_t faces = s.indices.size() / 3;
    out->assign(faces * 3, Float3(0.0f, 0.0f, 0.0f));
    std::vector<Float3> faceTangent(faces);
    auto pos = [&](const ObjIndex& i) { return Float3(d.positions[(size_t)i.v * 3], d.positions[(size_t)i.v * 3 + 1], d.positions[(size_t)i.v * 3 + 2]); };
    auto uv = [&](const ObjIndex& i) {
        Float2 t{ 0.0f, 0.0f };
        if (i.vt >= 0) { t.x = d.texcoords[(size_t)i.vt * 2]; t.y = d.texcoords[(size_t)i.vt * 2 + 1]; if (flipV) t.y = 1.0f - t.y; }
        return t;
    };
    for (size_t f = 0; f < faces; ++f) {
        const ObjIndex& a = s.indices[f * 3]; const ObjIndex& b = s.indices[f * 3 + 1]; const ObjIndex& c = s.indices[f * 3 + 2];
        const Float3 e1 = pos(b) - pos(a), e2 = pos(c) - pos(a);
        const Float2 ta = uv(a), tb = uv(b), tc = uv(c);
        const float du1 = tb.x - ta.x, dv1 = tb.y - ta.y, du2 = tc.x - ta.x, dv2 = tc.y - ta.y;
        const float r = du1 * dv2 - du2 * dv1;
        faceTangent[f] = r != 0.0f ? (e1 * dv2 - e2 * dv1) * (1.0f / r) : Float3(0.0f, 0.0f, 0.0f);
    }
    std::unordered_map<std::tuple<int, int, int>, Float3, IndexTripleHash> acc;
    for (size_t f = 0; f < faces; ++f)
        for (int k = 0; k < 3; ++k) {
            const ObjIndex& i = s.indices[f * 3 + k];
            Float3& t = acc[std::make_tuple(i.v, i.vn, i.vt)];
            t = t + faceTangent[f];
        }
    for (size_t f = 0; f < faces; ++f)
        for (int k = 0; k < 3; ++k) {
            const ObjIndex& i = s.indices[f * 3 + k];
            Float3 t = acc[std::make_tuple(i.v, i.vn, i.vt)];
            Float3 n(0.0f, 0.0f, 0.0f);
            if (i.vn >= 0) n = Float3(d.normals[(size_t)i.vn * 3], d.normals[(size_t)i.vn * 3 + 1], d.normals[(size_t)i.vn * 3 + 2]);
            const float nl = Length(n);
            if (nl > 0.0f) { n = n * (1.0f / nl); t = t - n * Dot(t, n); }
            const float tl = Length(t);
            (*out)[f * 3 + k] = tl > 0.0f ? t * (1.0f / tl) : Float3(0.0f, 0.0f, 0.0f);
        }
}

}  // namespace

bool ParseObjFile(const std::string& path, ObjData* out, std::string* err)
{
    std::ifstream in(path);
    if (!in) { if (err) *err = "cannot open " + path; return false; }
    const std::string dir = path.find_last_of('/') == std::string::npos ? std::string(".") : path.substr(0, path.find_last_of('/'));
    std::map<std::string, int> materialMap;
    ObjShape shape;
    std::string name;
    int material = -1;
    std::vector<std::vector<ObjIndex>> faces;   // current prim group
    std::vector<int> faceMaterials;
    auto exportGroup = [&]() {
        for (size_t i = 0; i < faces.size(); ++i) Triangulate(faces[i], out->positions, faceMaterials[i], &shape);
        bool had = !faces.empty();
        faces.clear(); faceMaterials.clear();
        shape.name = name;
        return had;
    };
    std::string line;
    while (std::getline(in, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        std::istringstream ss(line);
        std::string tag;
        if (!(ss >> tag)) continue;
        if (tag == "v") {
            double x = 0, y = 0, z = 0; ss >> x >> y >> z;
            out->positions.push_back((float)x); out->positions.push_back((float)y); out->positions.push_back((float)z);
        } else if (tag == "vn") {
            double x = 0, y = 0, z = 0; ss >> x >> y >> z;
            out->normals.push_back((float)x); out->normals.push_back((float)y); out->normals.push_back((float)z);
        } else if (tag == "vt") {
            double x = 0, y = 0; ss >> x >> y;
            out->texcoords.push_back((float)x); out->texcoords.push_back((float)y);
        } else if (tag == "f") {
            std::vector<ObjIndex> face;
            std::string tok;
            while (ss >> tok) {
                ObjIndex idx;
                if (!ParseCorner(tok, (int)out->positions.size() / 3, (int)out->normals.size() / 3, (int)out->texcoords.size() / 2, &idx)) {
                    if (err) *err = "bad face line: " + line;
                    return false;
                }
                face.push_back(idx);
            }
            faces.push_back(face);
            faceMaterials.push_back(material);
        } else if (tag == "usemtl") {
            std::string mname = Trim(line.substr(line.find("usemtl") + 6));
            auto it = materialMap.find(mname);
            int newId = it == materialMap.end() ? -1 : it->second;
            if (newId != material) {
                exportGroup();
                material = newId;
            }
        } else if (tag == "mtllib") {
            std::string file = Trim(line.substr(line.find("mtllib") + 6));
            const std::string full = (!file.empty() && file[0] == '/') ? file : dir + "/" + file;
            ParseMtl(full, &out->materials, &materialMap);
        } else if (tag == "g" || tag == "o") {
            exportGroup();
            if (!shape.indices.empty()) out->shapes.push_back(shape);
            shape = ObjShape();
            std::string rest = line.size() > 1 ? Trim(line.substr(1)) : std::string();
            name = rest;
        }
    }
    bool had = exportGroup();
    if (had || !shape.indices.empty()) out->shapes.push_back(shape);
    return true;
}

bool CreateMeshFromObjData(const ObjData& d, const ObjShape* shapes, uint32_t shapeCount, const SMeshProcessingParams& params, Mesh* mesh)
{
    if (d.normals.empty()) return false;
    Float4x4 normalTransform = Float4x4::Identity();
    if (params.applyTransform) normalTransform = Transpose(Inverse(params.transform));
    static const int kOriginal[3] = { 0, 1, 2 }, kChanged[3] = { 0, 2, 1 };
    const int* order = params.changeWindingOrder ? kChanged : kOriginal;
    std::unordered_map<CornerKey, uint32_t, CornerKeyHash> map;
    std::vector<Float3> tangents;
    for (uint32_t s = 0; s < shapeCount; ++s) {
        const ObjShape& shape = shapes[s];
        GenerateTangents(d, shape, params.flipTexcoordV, &tangents);
        const size_t faces = shape.indices.size() / 3;
        for (size_t f = 0; f < faces; ++f) {
            const int mat = shape.materialIds[f];
            mesh->materialIds.push_back(mat != -1 ? params.materialIndexBase + (uint32_t)mat : kInvalidMaterialId);
            for (int k = 0; k < 3; ++k) {
                const ObjIndex& idx = shape.indices[f * 3 + order[k]];
                if (idx.v < 0 || idx.vn < 0) return false;
                const Float3 tangent = tangents[f * 3 + order[k]];
                const CornerKey key{ idx.v, idx.vn, idx.vt, tangent.x, tangent.y, tangent.z };
                auto it = map.find(key);
                uint32_t vi;
                if (it != map.end()) {
                    vi = it->second;
                } else {
                    vi = (uint32_t)mesh->vertices.size();
                    dcrt_vertex vert{};
                    Float3 p(d.positions[(size_t)idx.v * 3], d.positions[(size_t)idx.v * 3 + 1], d.positions[(size_t)idx.v * 3 + 2]);
                    Float3 n(d.normals[(size_t)idx.vn * 3], d.normals[(size_t)idx.vn * 3 + 1], d.normals[(size_t)idx.vn * 3 + 2]);
                    Float3 t = tangent;
                    float u = 0.0f, v = 0.0f;
                    if (idx.vt >= 0) { u = d.texcoords[(size_t)idx.vt * 2]; v = d.texcoords[(size_t)idx.vt * 2 + 1]; }
                    if (params.flipTexcoordV) v = 1.0f - v;
                    if (params.applyTransform) {
                        p = TransformPoint(p, params.transform);
                        n = TransformNormal(n, normalTransform);
                        t = TransformNormal(t, normalTransform);
                    }
                    vert.position[0] = p.x; vert.position[1] = p.y; vert.position[2] = p.z;
                    vert.normal[0] = n.x; vert.normal[1] = n.y; vert.normal[2] = n.z;
                    vert.tangent[0] = t.x; vert.tangent[1] = t.y; vert.tangent[2] = t.z;
                    vert.texcoord[0] = u; vert.texcoord[1] = v;
                    mesh->vertices.push_back(vert);
                    map.emplace(key, vi);
                }
                mesh->indices.push_back(vi);
            }
        }
    }
    return true;
}

void TranslateObjMaterials(const ObjData& d, int32_t textureIndexBase, std::vector<SMaterial>* out, std::vector<std::string>* textureNames)
{
    std::unordered_map<std::string, int32_t> texIndex;
    auto getTex = [&](const std::string& name) {
        auto it = texIndex.find(name);
        if (it != texIndex.end()) return it->second;
        const int32_t idx = textureIndexBase + (int32_t)textureNames->size();
        texIndex[name] = idx;
        textureNames->push_back(name);
        return idx;
    };
    for (const ObjMaterial& m : d.materials) {   // WavefrontOBJLoading.cpp:305-338
        SMaterial s;
        s.albedo = Float3(m.diffuse[0], m.diffuse[1], m.diffuse[2]);
        s.roughness = m.roughness;
        s.ior = Float3(std::min(std::max(m.ior, 1.0f), kMaxMaterialIor), 1.0f, 1.0f);
        s.opacity = m.dissolve;
        s.k = Float3(1.0f, 1.0f, 1.0f);
        s.tiling = { 1.0f, 1.0f };
        s.type = EMaterialType::Plastic;
        s.multiscattering = false;
        s.isTwoSided = false;
        s.hasRoughnessTexture = false;
        s.internalScatteringMode = DCRT_INTERNAL_SCATTERING_IGNORE;
        s.name = m.name;
        s.albedoTextureIndex = m.diffuseTexname.empty() ? -1 : getTex(m.diffuseTexname);
        s.opacityTextureIndex = m.alphaTexname.empty() ? -1 : getTex(m.alphaTexname);
        out->push_back(s);
    }
}

// Binary PPM (P6 -> RGBA8 sRGB) / PGM (P5 -> R8) reader; WIC decoding (Texture.cpp) is Windows-only.
bool LoadTextureFile(const std::string& path, CTexture* out)
{
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    char magic[3] = { 0 };
    unsigned w = 0, h = 0, maxv = 0;
    bool ok = std::fscanf(f, "%2s %u %u %u", magic, &w, &h, &maxv) == 4 && maxv == 255 && w && h;
    if (ok) std::fgetc(f);
    if (ok && std::strcmp(magic, "P6") == 0) {
        std::vector<uint8_t> rgb((size_t)w * h * 3);
        ok = std::fread(rgb.data(), 1, rgb.size(), f) == rgb.size();
        out->pixels.resize((size_t)w * h * 4);
        for (size_t i = 0; i < (size_t)w * h; ++i) {
            out->pixels[i * 4] = rgb[i * 3]; out->pixels[i * 4 + 1] = rgb[i * 3 + 1]; out->pixels[i * 4 + 2] = rgb[i * 3 + 2]; out->pixels[i * 4 + 3] = 255;
        }
        out->format = DCRT_TEXTURE_FORMAT_RGBA8_SRGB;
    } else if (ok && std::strcmp(magic, "P5") == 0) {
        out->pixels.resize((size_t)w * h);
        ok = std::fread(out->pixels.data(), 1, out->pixels.size(), f) == out->pixels.size();
        out->format = DCRT_TEXTURE_FORMAT_R8_UNORM;
    } else {
        ok = false;
    }
    std::fclose(f);
    if (ok) { out->width = w; out->height = h; }
    else out->pixels.clear();
    return ok;
}

}  // namespace dcrt
