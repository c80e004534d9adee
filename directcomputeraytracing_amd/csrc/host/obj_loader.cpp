// obj_loader.cpp -- Wavefront OBJ/MTL loading for CScene
// (Source/WavefrontOBJLoading.cpp:155-465). The reference parses with tinyobjloader
// (/root/reference/tinyobjloader/tiny_obj_loader.h, LoadObj with triangulation) and
// generates tangents with MikkTSpace; both are parity-defining (vertex bits, vertex
// order, triangle order), so this parser restates the tinyobjloader behaviours the
// loader depends on -- its digit-by-digit number parsing, line/token rules, shape
// splitting on g/o/usemtl, ear-clipping triangulation and MTL defaults -- and
// tangent_space.cpp restates genTangSpaceDefault. tests/test_obj_pin.py checks the
// result bit for bit against the unmodified reference libraries built test-side
// (oracle/ref_obj/).
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

inline bool Blank(char c) { return c == ' ' || c == '\t'; }
inline bool LineEnd(char c) { return c == '\r' || c == '\n' || c == '\0'; }
inline bool Digit(char c) { return (unsigned)(c - '0') < 10u; }

// One line with tinyobjloader's safeGetline rules: "\n", "\r\n" and a lone "\r" end a
// line (tiny_obj_loader.h:730-762).
bool NextLine(std::istream& in, std::string* line)
{
    line->clear();
    std::streambuf* sb = in.rdbuf();
    if (sb->sgetc() == EOF) return false;
    for (;;) {
        const int c = sb->sbumpc();
        if (c == '\n' || c == EOF) return true;
        if (c == '\r') {
            if (sb->sgetc() == '\n') sb->sbumpc();
            return true;
        }
        line->push_back((char)c);
    }
}

// tryParseDouble (tiny_obj_loader.h:836-960): the integer digits accumulate as m*10 + d,
// fraction digit k adds d * 10^-k (a table for k < 8, pow beyond), an exponent e scales
// by ldexp(m * 5^e, e). Not correctly rounded, so it is restated rather than strtod.
bool ObjReal(const char* s, const char* end, double* out)
{
    if (s >= end) return false;
    static const double kFrac[8] = { 1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001 };
    double m = 0.0;
    int e10 = 0, digits = 0;
    char sign = '+', expSign = '+';
    const char* c = s;
    bool leadingDot = false;
    if (*c == '+' || *c == '-') {
        sign = *c++;
        leadingDot = c != end && *c == '.';
    } else if (*c == '.') {
        leadingDot = true;
    } else if (!Digit(*c)) {
        return false;
    }
    bool more = c != end;
    if (!leadingDot) {
        while (more && Digit(*c)) {
            m *= 10;
            m += (int)(*c - '0');
            ++c; ++digits;
            more = c != end;
        }
        if (digits == 0) return false;
    }
    if (more) {
        bool exponent = false;
        if (*c == '.') {
            ++c;
            int k = 1;
            more = c != end;
            while (more && Digit(*c)) {
                m += (int)(*c - '0') * (k < 8 ? kFrac[k] : std::pow(10.0, -k));
                ++k; ++c;
                more = c != end;
            }
            exponent = more && (*c == 'e' || *c == 'E');
        } else {
            exponent = *c == 'e' || *c == 'E';
        }
        if (exponent) {
            ++c;
            more = c != end;
            if (more && (*c == '+' || *c == '-')) expSign = *c++;
            else if (!Digit(*c)) return false;
            digits = 0;
            more = c != end;
            while (more && Digit(*c)) {
                e10 *= 10;
                e10 += (int)(*c - '0');
                ++c; ++digits;
                more = c != end;
            }
            e10 *= expSign == '+' ? 1 : -1;
            if (digits == 0) return false;
        }
    }
    *out = (sign == '+' ? 1 : -1) * (e10 ? std::ldexp(m * std::pow(5.0, e10), e10) : m);
    return true;
}

// parseReal: one blank-delimited token, the default when it does not parse
float TakeReal(const char** tok, double dflt = 0.0, bool* parsed = nullptr)
{
    *tok += std::strspn(*tok, " \t");
    const char* end = *tok + std::strcspn(*tok, " \t\r");
    double v = dflt;
    const bool ok = ObjReal(*tok, end, &v);
    if (parsed) *parsed = ok;
    *tok = end;
    return (float)v;
}

int TakeInt(const char** tok)
{
    *tok += std::strspn(*tok, " \t");
    const int v = std::atoi(*tok);
    *tok += std::strcspn(*tok, " \t\r");
    return v;
}

std::string TakeWord(const char** tok)
{
    *tok += std::strspn(*tok, " \t");
    const size_t n = std::strcspn(*tok, " \t\r");
    std::string w(*tok, n);
    *tok += n;
    return w;
}

// 1-based, negative = relative to the elements so far, 0 = error (fixIndex)
bool FixIndex(int idx, int n, int* out)
{
    if (idx > 0) { *out = idx - 1; return true; }
    if (idx < 0) { *out = n + idx; return true; }
    return false;
}

// "v", "v/vt", "v//vn", "v/vt/vn" (parseTriple)
bool TakeCorner(const char** tok, int nv, int nvn, int nvt, ObjIndex* out)
{
    ObjIndex r;
    if (!FixIndex(std::atoi(*tok), nv, &r.v)) return false;
    *tok += std::strcspn(*tok, "/ \t\r");
    if (**tok != '/') { *out = r; return true; }
    ++*tok;
    if (**tok == '/') {
        ++*tok;
        if (!FixIndex(std::atoi(*tok), nvn, &r.vn)) return false;
        *tok += std::strcspn(*tok, "/ \t\r");
        *out = r;
        return true;
    }
    if (!FixIndex(std::atoi(*tok), nvt, &r.vt)) return false;
    *tok += std::strcspn(*tok, "/ \t\r");
    if (**tok != '/') { *out = r; return true; }
    ++*tok;
    if (!FixIndex(std::atoi(*tok), nvn, &r.vn)) return false;
    *tok += std::strcspn(*tok, "/ \t\r");
    *out = r;
    return true;
}

bool PointInTriangle(const float* vx, const float* vy, float tx, float ty)   // pnpoly, 3 vertices
{
    bool c = false;
    for (int i = 0, j = 2; i < 3; j = i++)
        if (((vy[i] > ty) != (vy[j] > ty)) && (tx < (vx[j] - vx[i]) * (ty - vy[i]) / (vy[j] - vy[i]) + vx[i])) c = !c;
    return c;
}

// Ear clipping as tinyobjloader's exportGroupsToShape (tiny_obj_loader.h:1365-1598): a fan
// on convex faces; corners whose vertex index is out of range read as (0, 0).
void Triangulate(const std::vector<ObjIndex>& face, const std::vector<float>& v, int materialId, ObjShape* shape)
{
    const size_t n = face.size();
    if (n < 3) return;
    auto valid = [&](const ObjIndex& i, size_t axis) { return (size_t)i.v * 3 + axis < v.size(); };
    auto P = [&](const ObjIndex& i, size_t axis) { return v[(size_t)i.v * 3 + axis]; };
    size_t axes[2] = { 1, 2 };
    for (size_t k = 0; k < n; ++k) {
        const ObjIndex& a = face[k % n]; const ObjIndex& b = face[(k + 1) % n]; const ObjIndex& c = face[(k + 2) % n];
        if (!valid(a, 2) || !valid(b, 2) || !valid(c, 2)) continue;
        const float e0x = P(b, 0) - P(a, 0), e0y = P(b, 1) - P(a, 1), e0z = P(b, 2) - P(a, 2);
        const float e1x = P(c, 0) - P(b, 0), e1y = P(c, 1) - P(b, 1), e1z = P(c, 2) - P(b, 2);
        const float cx = std::fabs(e0y * e1z - e0z * e1y), cy = std::fabs(e0z * e1x - e0x * e1z), cz = std::fabs(e0x * e1y - e0y * e1x);
        const float eps = 1.1920929e-07f;
        if (cx > eps || cy > eps || cz > eps) {
            if (!(cx > cy && cx > cz)) { axes[0] = 0; if (cz > cx && cz > cy) axes[1] = 1; }
            break;
        }
    }
    float area = 0.0f;
    for (size_t k = 0; k < n; ++k) {
        const ObjIndex& a = face[k % n]; const ObjIndex& b = face[(k + 1) % n];
        if (!valid(a, axes[0]) || !valid(a, axes[1]) || !valid(b, axes[0]) || !valid(b, axes[1])) continue;
        area += (P(a, axes[0]) * P(b, axes[1]) - P(a, axes[1]) * P(b, axes[0])) * 0.5f;
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
            const bool ok = valid(ind[k], axes[0]) && valid(ind[k], axes[1]);
            vx[k] = ok ? P(ind[k], axes[0]) : 0.0f;
            vy[k] = ok ? P(ind[k], axes[1]) : 0.0f;
        }
        const float e0x = vx[1] - vx[0], e0y = vy[1] - vy[0], e1x = vx[2] - vx[1], e1y = vy[2] - vy[1];
        const float cross = e0x * e1y - e0y * e1x;
        if (cross * area < 0.0f) { guess += 1; continue; }
        bool overlap = false;
        for (size_t o = 3; o < np; ++o) {
            const ObjIndex& oi = rem[(guess + o) % np];
            if (!valid(oi, axes[0]) || !valid(oi, axes[1])) continue;
            if (PointInTriangle(vx, vy, P(oi, axes[0]), P(oi, axes[1]))) { overlap = true; break; }
        }
        if (overlap) { guess += 1; continue; }
        emit(ind[0], ind[1], ind[2]);
        rem.erase(rem.begin() + (long)((guess + 1) % np));
    }
    if (rem.size() == 3) emit(rem[0], rem[1], rem[2]);
}

// ParseTextureNameAndOption (tiny_obj_loader.h:1186-1270): options are skipped, the
// texture name is the rest of the line
bool TakeTextureName(const char* tok, std::string* name)
{
    bool found = false;
    auto opt = [&](const char* o) {
        const size_t n = std::strlen(o);
        return std::strncmp(tok, o, n) == 0 && Blank(tok[n]);
    };
    while (!LineEnd(*tok)) {
        tok += std::strspn(tok, " \t");
        if (opt("-blendu") || opt("-blendv")) { tok += 8; tok += std::strspn(tok, " \t"); tok += std::strcspn(tok, " \t\r"); }
        else if (opt("-clamp")) { tok += 7; tok += std::strspn(tok, " \t"); tok += std::strcspn(tok, " \t\r"); }
        else if (opt("-boost")) { tok += 7; TakeReal(&tok, 1.0); }
        else if (opt("-bm")) { tok += 4; TakeReal(&tok, 1.0); }
        else if (opt("-o") || opt("-s") || opt("-t")) { tok += 3; TakeReal(&tok); TakeReal(&tok); TakeReal(&tok); }
        else if (opt("-type")) { tok += 5; tok += std::strspn(tok, " \t"); tok += std::strcspn(tok, " \t\r"); }
        else if (opt("-texres")) { tok += 7; TakeInt(&tok); }
        else if (opt("-imfchan")) { tok += 9; tok += std::strspn(tok, " \t"); tok += std::strcspn(tok, " \t\r"); }
        else if (opt("-mm")) { tok += 4; TakeReal(&tok); TakeReal(&tok); }
        else if (opt("-colorspace")) { tok += 12; TakeWord(&tok); }
        else { *name = tok; tok += name->size(); found = true; }
    }
    return found;
}

// LoadMtl (tiny_obj_loader.h:1688-2077), the fields the OBJ material translation reads
// (WavefrontOBJLoading.cpp:305-338): Kd, Ni, Pr, d / Tr, map_Kd, map_d. A material is
// flushed at the next newmtl when it has a name, and always at the end of the file.
void ParseMtl(std::istream& in, std::vector<ObjMaterial>* mats, std::map<std::string, int>* index)
{
    ObjMaterial cur;
    bool hasD = false, hasTr = false, hasKd = false;
    std::string line;
    auto flush = [&]() {
        index->insert({ cur.name, (int)mats->size() });
        mats->push_back(cur);
    };
    while (NextLine(in, &line)) {
        line = line.substr(0, line.find_last_not_of(" \t") + 1);
        if (!line.empty() && line.back() == '\n') line.pop_back();
        if (!line.empty() && line.back() == '\r') line.pop_back();
        const char* tok = line.c_str();
        tok += std::strspn(tok, " \t");
        if (tok[0] == '\0' || tok[0] == '#') continue;
        if (std::strncmp(tok, "newmtl", 6) == 0 && Blank(tok[6])) {
            if (!cur.name.empty()) flush();
            cur = ObjMaterial();
            hasD = hasTr = false;
            cur.name = tok + 7;
        } else if (tok[0] == 'K' && tok[1] == 'd' && Blank(tok[2])) {
            tok += 2;
            for (int k = 0; k < 3; ++k) cur.diffuse[k] = TakeReal(&tok);
            hasKd = true;
        } else if (tok[0] == 'N' && tok[1] == 'i' && Blank(tok[2])) {
            tok += 2;
            cur.ior = TakeReal(&tok);
        } else if (tok[0] == 'd' && Blank(tok[1])) {
            tok += 1;
            cur.dissolve = TakeReal(&tok);
            hasD = true;
        } else if (tok[0] == 'T' && tok[1] == 'r' && Blank(tok[2])) {
            tok += 2;
            if (!hasD) cur.dissolve = 1.0f - TakeReal(&tok);
            hasTr = true;
        } else if (tok[0] == 'P' && tok[1] == 'r' && Blank(tok[2])) {
            tok += 2;
            cur.roughness = TakeReal(&tok);
        } else if (std::strncmp(tok, "map_Kd", 6) == 0 && Blank(tok[6])) {
            TakeTextureName(tok + 7, &cur.diffuseTexname);
            if (!hasKd) cur.diffuse[0] = cur.diffuse[1] = cur.diffuse[2] = 0.6f;
        } else if (std::strncmp(tok, "map_d", 5) == 0 && Blank(tok[5])) {
            cur.alphaTexname = tok + 6;
            TakeTextureName(tok + 6, &cur.alphaTexname);
        }
    }
    (void)hasTr;
    flush();
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

// Tangents for one shape's triangles through MikkTSpace's interface view of the mesh
// (WavefrontOBJLoading.cpp:102-153): raw OBJ positions and normals, uv with the V flip,
// a missing uv reads (0, 0).
bool ShapeTangents(const ObjData& d, const ObjShape& s, bool flipV, std::vector<Float3>* out)
{
    const size_t corners = s.indices.size();
    std::vector<Float3> pos(corners), nrm(corners), uvw(corners);
    for (size_t c = 0; c < corners; ++c) {
        const ObjIndex& i = s.indices[c];
        pos[c] = Float3(d.positions[(size_t)i.v * 3], d.positions[(size_t)i.v * 3 + 1], d.positions[(size_t)i.v * 3 + 2]);
        nrm[c] = Float3(d.normals[(size_t)i.vn * 3], d.normals[(size_t)i.vn * 3 + 1], d.normals[(size_t)i.vn * 3 + 2]);
        float u = 0.0f, v = 0.0f;
        if (i.vt != -1) {
            u = d.texcoords[(size_t)i.vt * 2];
            v = d.texcoords[(size_t)i.vt * 2 + 1];
            if (flipV) v = 1.0f - v;
        }
        uvw[c] = Float3(u, v, 1.0f);
    }
    return GenerateMikkTangents(pos, nrm, uvw, out);
}

}  // namespace

bool ParseObjFile(const std::string& path, ObjData* out, std::string* err)
{
    std::ifstream in(path, std::ios::binary);
    if (!in) { if (err) *err = "cannot open " + path; return false; }
    // MTL search path: the OBJ's directory (WavefrontOBJLoading.cpp:412), '/' appended
    std::string baseDir = path.find_last_of('/') == std::string::npos ? std::string() : path.substr(0, path.find_last_of('/'));
    if (!baseDir.empty() && baseDir.back() != '/') baseDir += '/';
    std::map<std::string, int> materialMap;
    ObjShape shape;
    std::string name;
    int material = -1;
    std::vector<std::vector<ObjIndex>> faces;   // current prim group
    std::vector<int> faceMaterials;
    size_t otherPrims = 0;                      // l / p elements of the current prim group
    bool shapeHasOther = false;                 // the shape holds exported l / p elements
    auto exportGroup = [&]() {                  // exportGroupsToShape: false for an empty group
        if (faces.empty() && otherPrims == 0) return false;
        shape.name = name;
        shapeHasOther = shapeHasOther || otherPrims != 0;
        for (size_t i = 0; i < faces.size(); ++i) Triangulate(faces[i], out->positions, faceMaterials[i], &shape);
        return true;
    };
    auto clearGroup = [&]() { faces.clear(); faceMaterials.clear(); otherPrims = 0; };
    std::string line;
    while (NextLine(in, &line)) {
        if (!line.empty() && line.back() == '\n') line.pop_back();
        if (!line.empty() && line.back() == '\r') line.pop_back();
        const char* tok = line.c_str();
        tok += std::strspn(tok, " \t");
        if (tok[0] == '\0' || tok[0] == '#') continue;
        const int nv = (int)(out->positions.size() / 3), nvn = (int)(out->normals.size() / 3), nvt = (int)(out->texcoords.size() / 2);
        if (tok[0] == 'v' && Blank(tok[1])) {
            tok += 2;
            for (int k = 0; k < 3; ++k) out->positions.push_back(TakeReal(&tok));
            continue;
        }
        if (tok[0] == 'v' && tok[1] == 'n' && Blank(tok[2])) {
            tok += 3;
            for (int k = 0; k < 3; ++k) out->normals.push_back(TakeReal(&tok));
            continue;
        }
        if (tok[0] == 'v' && tok[1] == 't' && Blank(tok[2])) {
            tok += 3;
            for (int k = 0; k < 2; ++k) out->texcoords.push_back(TakeReal(&tok));
            continue;
        }
        if ((tok[0] == 'l' || tok[0] == 'p') && Blank(tok[1])) {
            tok += 2;
            while (!LineEnd(tok[0])) {
                ObjIndex idx;
                if (!TakeCorner(&tok, nv, nvn, nvt, &idx)) {
                    if (err) *err = "bad line/point element: " + line;
                    return false;
                }
                tok += std::strspn(tok, " \t\r");
            }
            ++otherPrims;
            continue;
        }
        if (tok[0] == 'f' && Blank(tok[1])) {
            tok += 2;
            tok += std::strspn(tok, " \t");
            std::vector<ObjIndex> face;
            while (!LineEnd(tok[0])) {
                ObjIndex idx;
                if (!TakeCorner(&tok, nv, nvn, nvt, &idx)) {
                    if (err) *err = "bad face line: " + line;
                    return false;
                }
                face.push_back(idx);
                tok += std::strspn(tok, " \t\r");
            }
            faces.push_back(std::move(face));
            faceMaterials.push_back(material);
            continue;
        }
        if (std::strncmp(tok, "usemtl", 6) == 0) {
            tok += 6;
            const std::string mname = TakeWord(&tok);
            auto it = materialMap.find(mname);
            const int newId = it == materialMap.end() ? -1 : it->second;
            if (newId != material) {
                exportGroup();
                faces.clear(); faceMaterials.clear();
                material = newId;
            }
            continue;
        }
        if (std::strncmp(tok, "mtllib", 6) == 0 && Blank(tok[6])) {
            std::stringstream names(std::string(tok + 7));
            std::string file;
            while (std::getline(names, file, ' ')) {
                // MaterialFileReader: the search path joined with the name as written
                const std::string full = baseDir.empty() ? file : baseDir + file;
                std::ifstream mtl(full, std::ios::binary);
                if (mtl) { ParseMtl(mtl, &out->materials, &materialMap); break; }
            }
            continue;
        }
        if (tok[0] == 'g' && Blank(tok[1])) {
            exportGroup();
            if (!shape.indices.empty()) out->shapes.push_back(shape);
            shape = ObjShape();
            shapeHasOther = false;
            clearGroup();
            std::vector<std::string> names;
            while (!LineEnd(tok[0])) {
                names.push_back(TakeWord(&tok));
                tok += std::strspn(tok, " \t\r");
            }
            name.clear();
            for (size_t i = 1; i < names.size(); ++i) name += (i > 1 ? " " : "") + names[i];
            continue;
        }
        if (tok[0] == 'o' && Blank(tok[1])) {
            exportGroup();
            if (!shape.indices.empty() || shapeHasOther) out->shapes.push_back(shape);
            clearGroup();
            shape = ObjShape();
            shapeHasOther = false;
            name = tok + 2;
            continue;
        }
        // vw, t, s and unknown statements carry nothing the loader reads
    }
    const bool exported = exportGroup();
    if (exported || !shape.indices.empty()) out->shapes.push_back(shape);
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
        // a corner without position or normal fails the mesh (:212-213); the reference
        // reads such corners' attributes out of bounds in MikkTSpace first, so they and
        // out-of-range indices are refused before any attribute is read -- a texcoord index
        // too (only -1 means "none": a relative index reaching before the first texcoord
        // resolves to another negative value, which the reference reads out of bounds)
        for (const ObjIndex& idx : shape.indices)
            if (idx.v < 0 || idx.vn < 0 || (size_t)idx.v * 3 + 2 >= d.positions.size() ||
                (size_t)idx.vn * 3 + 2 >= d.normals.size() ||
                (idx.vt != -1 && (idx.vt < 0 || (size_t)idx.vt * 2 + 1 >= d.texcoords.size())))
                return false;
        // a shape MikkTSpace refuses (no triangles) is skipped (WavefrontOBJLoading.cpp:195-199)
        if (!ShapeTangents(d, shape, params.flipTexcoordV, &tangents)) continue;
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
