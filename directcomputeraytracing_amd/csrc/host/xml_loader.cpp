// xml_loader.cpp -- the Mitsuba 3 XML subset CScene::LoadFromXMLFile reads
// (Source/SceneXMLLoading.cpp), restated: a small XML parser, the "value graph"
// of objects/fields/nested objects/refs/defaults (:247-581), BSDF translation
// (:625-923), and the scene walk over integrator / sensor / film / rfilter /
// bsdf / shape (obj, rectangle) / emitter (area, constant, directional)
// (:960-1512). Quirks of the reference are kept and marked "(quirk)".
#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "scene.h"

namespace dcrt {

void SetLastError(const std::string& s);

namespace {

constexpr float kMaxMaterialEta = 7.0f;   // Constants.h:4
constexpr float kMaxMaterialK = 9.5f;     // Constants.h:5
constexpr float kPi = 3.141592654f;       // XM_PI

// ------------------------------------------------------------------ XML DOM
struct XNode {
    std::string name;
    std::vector<std::pair<std::string, std::string>> attrs;
    std::vector<std::unique_ptr<XNode>> children;
    const std::string* Attr(const char* n) const
    {
        for (const auto& a : attrs)
            if (a.first == n) return &a.second;
        return nullptr;
    }
};

class XmlParser {
public:
    explicit XmlParser(const std::string& t) : s_(t) {}
    bool Parse(XNode* doc)
    {
        while (true) {
            SkipMisc();
            if (p_ >= s_.size()) return true;
            if (s_[p_] != '<') return Fail("unexpected text at top level");
            auto n = std::make_unique<XNode>();
            if (!Element(n.get())) return false;
            doc->children.push_back(std::move(n));
        }
    }
    std::string error;

private:
    bool Fail(const char* m)
    {
        error = std::string(m) + " at offset " + std::to_string(p_);
        return false;
    }
    void SkipWs()
    {
        while (p_ < s_.size() && (s_[p_] == ' ' || s_[p_] == '\t' || s_[p_] == '\n' || s_[p_] == '\r')) ++p_;
    }
    bool StartsWith(const char* t) const { return s_.compare(p_, std::strlen(t), t) == 0; }
    // comments, processing instructions, doctype, and character data between tags
    void SkipMisc()
    {
        while (p_ < s_.size()) {
            SkipWs();
            if (StartsWith("<!--")) {
                const size_t e = s_.find("-->", p_ + 4);
                p_ = e == std::string::npos ? s_.size() : e + 3;
            } else if (StartsWith("<?")) {
                const size_t e = s_.find("?>", p_ + 2);
                p_ = e == std::string::npos ? s_.size() : e + 2;
            } else if (StartsWith("<!")) {
                const size_t e = s_.find('>', p_ + 2);
                p_ = e == std::string::npos ? s_.size() : e + 1;
            } else if (p_ < s_.size() && s_[p_] != '<') {
                const size_t e = s_.find('<', p_);
                p_ = e == std::string::npos ? s_.size() : e;
            } else {
                return;
            }
        }
    }
    static bool NameChar(char c) { return std::isalnum((unsigned char)c) || c == '_' || c == '-' || c == ':' || c == '.'; }
    std::string Name()
    {
        const size_t b = p_;
        while (p_ < s_.size() && NameChar(s_[p_])) ++p_;
        return s_.substr(b, p_ - b);
    }
    bool Element(XNode* n)
    {
        ++p_;   // '<'
        n->name = Name();
        if (n->name.empty()) return Fail("expected element name");
        while (true) {
            SkipWs();
            if (p_ >= s_.size()) return Fail("unterminated tag");
            if (StartsWith("/>")) { p_ += 2; return true; }
            if (s_[p_] == '>') { ++p_; break; }
            std::string an = Name();
            if (an.empty()) return Fail("expected attribute name");
            SkipWs();
            if (p_ >= s_.size() || s_[p_] != '=') return Fail("expected '='");
            ++p_;
            SkipWs();
            if (p_ >= s_.size() || (s_[p_] != '"' && s_[p_] != '\'')) return Fail("expected quoted attribute value");
            const char q = s_[p_++];
            const size_t e = s_.find(q, p_);
            if (e == std::string::npos) return Fail("unterminated attribute value");
            // (quirk) the reference parses with rapidxml::parse_non_destructive
            // (SceneXMLLoading.cpp:1056): no entity translation, "&amp;" stays as written
            n->attrs.emplace_back(an, s_.substr(p_, e - p_));
            p_ = e + 1;
        }
        while (true) {
            SkipMisc();
            if (p_ >= s_.size()) return Fail("missing closing tag");
            if (StartsWith("</")) {
                p_ += 2;
                const std::string cn = Name();
                SkipWs();
                if (cn != n->name || p_ >= s_.size() || s_[p_] != '>') return Fail("mismatched closing tag");
                ++p_;
                return true;
            }
            auto c = std::make_unique<XNode>();
            if (!Element(c.get())) return false;
            n->children.push_back(std::move(c));
        }
    }
    const std::string& s_;
    size_t p_ = 0;
};

// The element / attribute tree as the reference's walk sees it (rapidxml element nodes in
// document order, attributes in order): "E<name>\n", "A<name>=<value>\n" per attribute,
// the children, "/\n". tests/test_xml_pin.py compares it with the reference's rapidxml.
void DumpTree(const XNode& n, std::string* out)
{
    for (const auto& c : n.children) {
        *out += "E" + c->name + "\n";
        for (const auto& a : c->attrs) *out += "A" + a.first + "=" + a.second + "\n";
        DumpTree(*c, out);
        *out += "/\n";
    }
}

// ------------------------------------------------------------------ value graph (:13-581)
enum class VT { Float, Integer, Boolean, String, Vector /* = RGB */, Matrix, Object };

struct Value {
    VT type = VT::Float;
    float f = 0.0f;
    int32_t i = 0;
    bool b = false;
    std::string s;
    Float3 v;
    Float4x4 m = Float4x4::Identity();
    std::string tag;                                          // element name of an object
    std::unordered_map<std::string, Value*> fields;
    std::vector<std::pair<std::string, Value*>> nested;

    Value* Field(const std::string& n) const
    {
        auto it = fields.find(n);
        return it == fields.end() ? nullptr : it->second;
    }
    Value* FirstNested(const std::string& n) const
    {
        for (const auto& p : nested)
            if (p.first == n) return p.second;
        return nullptr;
    }
    // GetObjectField<T>: the default unless the field exists with the matching type
    float GetFloat(const char* n, float d) const { Value* x = Field(n); return x && x->type == VT::Float ? x->f : d; }
    int32_t GetInt(const char* n, int32_t d) const { Value* x = Field(n); return x && x->type == VT::Integer ? x->i : d; }
    bool GetBool(const char* n, bool d) const { Value* x = Field(n); return x && x->type == VT::Boolean ? x->b : d; }
    std::string GetString(const char* n, const std::string& d) const { Value* x = Field(n); return x && x->type == VT::String ? x->s : d; }
    Float3 GetVec(const char* n, Float3 d) const { Value* x = Field(n); return x && x->type == VT::Vector ? x->v : d; }
    // SValue::m_Float read whatever the value holds -- the reference's unchecked reads (alpha :888,
    // aperture_radius :1241, focus_distance :1244) see the union's first word: an integer's or a
    // boolean's bits (SValue() zeroes the word, m_Boolean sets its low byte), a vector's x, a
    // matrix's _11. (A string's or an object's first word is a pointer: undefined, 0 here.)
    float UnionFloat() const
    {
        uint32_t w = 0;
        switch (type) {
        case VT::Float: return f;
        case VT::Integer: std::memcpy(&w, &i, 4); break;
        case VT::Boolean: w = b ? 1u : 0u; break;
        case VT::Vector: return v.x;
        case VT::Matrix: return m.m[0][0];
        default: return 0.0f;
        }
        float r;
        std::memcpy(&r, &w, 4);
        return r;
    }
};

// strncmp(a, literal, len(a)) == 0 as the reference writes its keyword tests: a
// prefix of the literal matches (quirk)
bool KeywordIs(const std::string& a, const char* lit) { return std::strncmp(a.c_str(), lit, a.size()) == 0; }

std::vector<std::string> Split(const std::string& s, char d)   // SplitByDelimeter (:213-230)
{
    std::vector<std::string> out;
    size_t i = 0;
    while (i < s.size()) {
        size_t e = s.find(d, i);
        if (e == std::string::npos) e = s.size();
        out.push_back(s.substr(i, e - i));
        i = e + 1;
    }
    return out;
}

class Graph {
public:
    std::vector<std::unique_ptr<Value>> pool;
    std::unordered_map<std::string, Value*> objects;          // id -> object (first definition wins)
    std::unordered_map<std::string, std::string> defaults;    // <default name= value=>
    std::string error;

    Value* New()
    {
        pool.push_back(std::make_unique<Value>());
        return pool.back().get();
    }
    bool Eval(const std::string& in, std::string* out)   // TryEvaluateValueString (:193-211)
    {
        if (!in.empty() && in[0] == '$') {
            auto it = defaults.find(in.substr(1));
            if (it == defaults.end()) {
                error = "unknown default parameter " + in;
                return false;
            }
            *out = it->second;
            return true;
        }
        *out = in;
        return true;
    }
    bool IsObjectTag(const std::string& n) const
    {
        static const char* tags[] = { "scene", "integrator", "sensor", "sampler", "film", "bsdf", "rfilter", "emitter", "shape", "texture" };
        for (const char* t : tags)
            if (n == t) return true;
        return false;
    }
    bool IsValueTag(const std::string& n) const
    {
        static const char* tags[] = { "float", "integer", "boolean", "string", "point", "vector", "rgb" };
        for (const char* t : tags)
            if (n == t) return true;
        return false;
    }
    void Attach(Value* parent, const XNode& node, Value* v)
    {
        const std::string* nm = node.Attr("name");
        if (nm) parent->fields.insert({ *nm, v });
        else parent->nested.emplace_back(node.name, v);
    }
    void RegisterId(const XNode& node, Value* v)
    {
        const std::string* id = node.Attr("id");
        if (!id) return;
        if (!objects.count(*id)) objects[*id] = v;
        else std::fprintf(stderr, "dcrt: duplicated id '%s'\n", id->c_str());
        Value* idv = New();
        idv->type = VT::String;
        idv->s = *id;
        v->fields.insert({ "id", idv });
    }
    bool Children(const XNode& node, Value* parent);
    bool Build(const XNode& sceneNode, Value** scene)
    {
        const std::string* ver = sceneNode.Attr("version");
        if (!ver) { error = "cannot find version attribute at the scene tag"; return false; }
        const std::vector<std::string> parts = Split(*ver, '.');
        if (parts.size() != 3) { error = "unsupported scene version format " + *ver; return false; }
        if (std::atoi(parts[0].c_str()) < 3) { error = "unsupported scene version " + *ver; return false; }
        Value* v = New();
        v->type = VT::Object;
        v->tag = "scene";
        *scene = v;
        return Children(sceneNode, v);
    }
};

bool Graph::Children(const XNode& node, Value* parent)
{
    for (const auto& cp : node.children) {
        const XNode& c = *cp;
        if (IsObjectTag(c.name)) {
            Value* v = New();
            v->type = VT::Object;
            v->tag = c.name;
            Attach(parent, c, v);
            RegisterId(c, v);
            if (const std::string* t = c.Attr("type")) {
                Value* tv = New();
                tv->type = VT::String;
                if (!Eval(*t, &tv->s)) return false;
                v->fields.insert({ "type", tv });
            }
            if (!Children(c, v)) return false;
        } else if (c.name == "transform") {
            Value* v = New();
            v->type = VT::Matrix;
            v->tag = c.name;
            Attach(parent, c, v);
            RegisterId(c, v);
            for (const auto& mp : c.children) {
                if (mp->name != "matrix") {
                    std::fprintf(stderr, "dcrt: unsupported child tag for transform '%s'\n", mp->name.c_str());
                    continue;
                }
                const std::string* val = mp->Attr("value");
                if (!val) { std::fprintf(stderr, "dcrt: expect value attribute for matrix\n"); continue; }
                std::string ev;
                if (!Eval(*val, &ev)) return false;
                const std::vector<std::string> nums = Split(ev, ' ');
                if (nums.size() != 16) { error = "unrecognized matrix value '" + ev + "'"; return false; }
                // Mitsuba: row-major, column vectors -> row-vector convention (transpose),
                // then right-handed -> left-handed by negating the x output (:377-389)
                for (int r = 0; r < 4; ++r)
                    for (int k = 0; k < 4; ++k) v->m.m[k][r] = (float)std::atof(nums[r * 4 + k].c_str());
                for (int r = 0; r < 4; ++r) v->m.m[r][0] = -v->m.m[r][0];
            }
        } else if (c.name == "ref") {
            const std::string* id = c.Attr("id");
            if (!id) { error = "expect id attribute in the ref tag"; return false; }
            auto it = objects.find(*id);
            if (it == objects.end()) {
                std::fprintf(stderr, "dcrt: id '%s' not found\n", id->c_str());
                continue;
            }
            if (const std::string* nm = c.Attr("name")) parent->fields.insert({ *nm, it->second });
            else parent->nested.emplace_back(it->second->tag, it->second);
        } else if (IsValueTag(c.name)) {
            const std::string* nm = c.Attr("name");
            if (!nm) { error = "expect a name attribute from tag '" + c.name + "'"; return false; }
            const std::string* val = c.Attr("value");
            if (!val) { error = "expect a value attribute"; return false; }
            Value* v = New();
            parent->fields.insert({ *nm, v });
            std::string ev;
            if (!Eval(*val, &ev)) return false;
            v->s = ev;    // raw text, also for non-string types (focal_length below)
            if (c.name == "integer") {
                v->type = VT::Integer;
                v->i = (int32_t)std::atoi(ev.c_str());
            } else if (c.name == "float") {
                v->type = VT::Float;
                v->f = (float)std::atof(ev.c_str());
            } else if (c.name == "boolean") {
                v->type = VT::Boolean;
                if (KeywordIs(ev, "false")) v->b = false;
                else if (KeywordIs(ev, "true")) v->b = true;
                else { error = "unrecognized boolean value"; return false; }
            } else if (c.name == "string") {
                v->type = VT::String;
            } else {   // point, vector, rgb
                v->type = VT::Vector;
                const std::vector<std::string> xyz = Split(ev, ',');
                if (xyz.size() != 3) { error = "unrecognized " + c.name + " value '" + ev + "'"; return false; }
                v->v = Float3((float)std::atof(xyz[0].c_str()), (float)std::atof(xyz[1].c_str()), (float)std::atof(xyz[2].c_str()));
            }
        } else if (c.name == "default") {
            const std::string* nm = c.Attr("name");
            const std::string* val = c.Attr("value");
            if (nm && val) defaults.insert({ *nm, *val });
        } else {
            std::fprintf(stderr, "dcrt: unsupported tag name \"%s\"\n", c.name.c_str());
        }
    }
    return true;
}

// ------------------------------------------------------------------ materials (:589-923)
enum class XMat { Unsupported, Diffuse, RoughDiffuse, Dielectric, ThinDielectric, RoughDielectric, Conductor, RoughConductor,
                  Plastic, RoughPlastic, Twosided, Mask };

XMat MaterialKind(const std::string& t)
{
    static const std::pair<const char*, XMat> kinds[] = {
        { "diffuse", XMat::Diffuse }, { "roughdiffuse", XMat::RoughDiffuse }, { "dielectric", XMat::Dielectric },
        { "thindielectric", XMat::ThinDielectric }, { "roughdielectric", XMat::RoughDielectric }, { "conductor", XMat::Conductor },
        { "roughconductor", XMat::RoughConductor }, { "plastic", XMat::Plastic }, { "roughplastic", XMat::RoughPlastic },
        { "twosided", XMat::Twosided }, { "mask", XMat::Mask } };
    for (const auto& k : kinds)
        if (t == k.first) return k.second;
    return XMat::Unsupported;
}

float ClampRange(const char* what, float v, float lo, float hi)
{
    if (v < lo || v > hi) {
        std::fprintf(stderr, "dcrt: %s %f is out of valid range, clamped to [%f, %f]\n", what, v, lo, hi);
        v = std::clamp(v, lo, hi);
    }
    return v;
}

struct MaterialContext {
    std::string scenePath;
    std::vector<SMaterial>* materials;
    uint32_t textureIndexBase;
    std::unordered_map<const Value*, uint32_t> bsdfToId;
    std::unordered_map<const Value*, uint32_t> textureToIndex;
    std::vector<std::pair<std::string, std::string>> textures;   // (filename, id)
    uint32_t unnamedTextures = 0;

    std::string Absolute(const std::string& f) const
    {
        if (!f.empty() && f[0] == '/') return f;
        const size_t slash = scenePath.find_last_of('/');
        return (slash == std::string::npos ? std::string(".") : scenePath.substr(0, slash)) + "/" + f;
    }
    int32_t GetOrAddTexture(const Value* v)   // :548-587
    {
        const std::string type = v->GetString("type", "");
        if (!KeywordIs(type, "bitmap")) {
            std::fprintf(stderr, "dcrt: unsupported texture type '%s'\n", type.c_str());
            return -1;
        }
        auto it = textureToIndex.find(v);
        if (it != textureToIndex.end()) return (int32_t)it->second;
        const uint32_t idx = textureIndexBase + (uint32_t)textureToIndex.size();
        textureToIndex.insert({ v, idx });
        std::string id;
        if (Value* idv = v->Field("id")) id = idv->s;
        else {
            char buf[32];
            std::snprintf(buf, sizeof(buf), "Texture%03u", unnamedTextures++);
            id = buf;
        }
        textures.emplace_back(Absolute(v->GetString("filename", "")), id);
        return (int32_t)idx;
    }
    bool Translate(const Value& bsdf, SMaterial* m, bool twoSided, bool isMask);
    bool CreateAndAdd(const Value& bsdf, uint32_t* id)
    {
        SMaterial m;
        if (!Translate(bsdf, &m, false, false)) return false;
        *id = (uint32_t)materials->size();
        materials->push_back(m);
        bsdfToId.insert({ &bsdf, *id });
        return true;
    }
};

bool MaterialContext::Translate(const Value& bsdf, SMaterial* m, bool twoSided, bool isMask)
{
    Value* typeValue = bsdf.Field("type");
    if (!typeValue) { std::fprintf(stderr, "dcrt: cannot obtain bsdf type\n"); return false; }
    const XMat kind = MaterialKind(typeValue->s);
    if (Value* idv = bsdf.Field("id")) m->name = idv->s;
    if (kind == XMat::Twosided || kind == XMat::Mask) {
        if (kind == XMat::Mask) {
            float opacity = 0.5f;
            int32_t opacityTexture = -1;
            if (Value* ov = bsdf.Field("opacity")) {
                if (ov->type == VT::Float) opacity = ov->f;
                else if (ov->type == VT::Object) opacityTexture = GetOrAddTexture(ov);
                else std::fprintf(stderr, "dcrt: unsupported opacity type\n");
            }
            m->opacity = opacityTexture == -1 ? opacity : 1.0f;
            m->opacityTextureIndex = opacityTexture;
        }
        Value* child = bsdf.FirstNested("bsdf");
        if (!child) { std::fprintf(stderr, "dcrt: cannot find child BSDF inside a nested BSDF\n"); return false; }
        return Translate(*child, m, kind == XMat::Twosided || twoSided, kind == XMat::Mask || isMask);
    }
    EMaterialType target = EMaterialType::Diffuse;
    bool dielectricIor = false, conductorIor = false, rough = false, diffuseReflectance = false;
    switch (kind) {
    case XMat::Diffuse: diffuseReflectance = true; break;
    case XMat::RoughDiffuse: diffuseReflectance = true; rough = true; break;
    case XMat::Dielectric: dielectricIor = true; target = EMaterialType::Dielectric; break;
    case XMat::ThinDielectric: dielectricIor = true; target = EMaterialType::ThinDielectric; break;
    case XMat::RoughDielectric: dielectricIor = true; rough = true; target = EMaterialType::Dielectric; break;
    case XMat::Conductor: conductorIor = true; target = EMaterialType::Conductor; break;
    case XMat::RoughConductor: conductorIor = true; rough = true; target = EMaterialType::Conductor; break;
    case XMat::Plastic: dielectricIor = true; diffuseReflectance = true; target = EMaterialType::Plastic; break;
    case XMat::RoughPlastic: dielectricIor = true; diffuseReflectance = true; rough = true; target = EMaterialType::Plastic; break;
    default: std::fprintf(stderr, "dcrt: unsupported material type '%s', assigning default values\n", typeValue->s.c_str()); break;
    }
    m->albedo = Float3(0.0f, 0.0f, 0.0f);
    m->roughness = 0.0f;
    m->ior = Float3(1.0f, 1.0f, 1.0f);
    m->k = Float3(1.0f, 1.0f, 1.0f);
    m->tiling = Float2{ 1.0f, 1.0f };
    m->type = target;
    m->albedoTextureIndex = -1;
    m->multiscattering = false;   // set only by the UI (ImGui.cpp:625)
    m->isTwoSided = twoSided;
    m->hasRoughnessTexture = false;
    m->internalScatteringMode = DCRT_INTERNAL_SCATTERING_MULTIPLE;
    if (!isMask) {
        m->opacity = 1.0f;
        m->opacityTextureIndex = -1;
    }
    if (target == EMaterialType::Plastic)
        m->internalScatteringMode = bsdf.GetBool("nonlinear", false) ? DCRT_INTERNAL_SCATTERING_MULTIPLE : DCRT_INTERNAL_SCATTERING_SINGLE;
    if (rough) {
        Value* a = bsdf.Field("alpha");
        const float alpha = a ? a->UnionFloat() : 0.1f;
        m->roughness = std::sqrt(alpha);
    }
    if (dielectricIor) {
        float intIor = 1.49f, extIor = 1.000277f;
        if (Value* v = bsdf.Field("int_ior")) {
            if (v->type == VT::Float) intIor = v->f;
            else std::fprintf(stderr, "dcrt: non-float IOR value is not supported\n");
        }
        if (Value* v = bsdf.Field("ext_ior")) {
            if (v->type == VT::Float) extIor = v->f;
            else std::fprintf(stderr, "dcrt: non-float IOR value is not supported\n");
        }
        m->ior.x = intIor / extIor;
    } else if (conductorIor) {
        Float3 eta(0.0f, 0.0f, 0.0f);
        float extEta = 1.000277f;
        if (Value* v = bsdf.Field("eta")) {
            if (v->type == VT::Vector) eta = v->v;
            else std::fprintf(stderr, "dcrt: non-RGB eta value is not supported\n");
        }
        if (Value* v = bsdf.Field("ext_eta")) {
            if (v->type == VT::Float) extEta = v->f;
            else std::fprintf(stderr, "dcrt: non-float ext_eta value is not supported\n");
        }
        m->ior = Float3(eta.x / extEta, eta.y / extEta, eta.z / extEta);
        Float3 k(1.0f, 1.0f, 1.0f);
        if (Value* v = bsdf.Field("k")) {
            if (v->type == VT::Vector) k = v->v;
            else std::fprintf(stderr, "dcrt: non-RGB k value is not supported\n");
        }
        m->k = k;
    }
    if (diffuseReflectance) {
        Float3 albedo(0.5f, 0.5f, 0.5f);
        int32_t tex = -1;
        if (Value* v = bsdf.Field(!dielectricIor ? "reflectance" : "diffuse_reflectance")) {
            if (v->type == VT::Vector) albedo = v->v;
            else if (v->type == VT::Object) tex = GetOrAddTexture(v);
            else std::fprintf(stderr, "dcrt: unsupported diffuse reflectance type\n");
        }
        m->albedo = tex == -1 ? albedo : Float3(1.0f, 1.0f, 1.0f);
        m->albedoTextureIndex = tex;
    }
    const bool conductor = m->type == EMaterialType::Conductor;
    const float minIor = conductor ? 0.0f : 1.0f, maxIor = conductor ? kMaxMaterialEta : kMaxMaterialIor;
    m->ior.x = ClampRange("Material IOR.x", m->ior.x, minIor, maxIor);
    m->ior.y = ClampRange("Material IOR.y", m->ior.y, minIor, maxIor);
    m->ior.z = ClampRange("Material IOR.z", m->ior.z, minIor, maxIor);
    m->k.x = ClampRange("Material K.x", m->k.x, 0.0f, kMaxMaterialK);
    m->k.y = ClampRange("Material K.y", m->k.y, 0.0f, kMaxMaterialK);
    m->k.z = ClampRange("Material K.z", m->k.z, 0.0f, kMaxMaterialK);
    return true;
}

}  // namespace

bool DumpXmlTree(const std::string& path, std::string* out)
{
    std::ifstream in(path, std::ios::binary);
    if (!in) { SetLastError("cannot open " + path); return false; }
    std::stringstream ss;
    ss << in.rdbuf();
    const std::string text = ss.str();
    XNode doc;
    XmlParser parser(text);
    if (!parser.Parse(&doc)) { SetLastError("XML parse error in " + path + ": " + parser.error); return false; }
    out->clear();
    DumpTree(doc, out);
    return true;
}

// CScene::LoadFromXMLFile (SceneXMLLoading.cpp:960-1512)
bool LoadMitsubaXML(CScene* scene, const std::string& path)
{
    std::ifstream in(path, std::ios::binary);
    if (!in) { SetLastError("cannot open " + path); return false; }
    std::stringstream ss;
    ss << in.rdbuf();
    const std::string text = ss.str();
    XNode doc;
    XmlParser parser(text);
    if (!parser.Parse(&doc)) { SetLastError("XML parse error in " + path + ": " + parser.error); return false; }
    const XNode* sceneNode = nullptr;
    for (const auto& c : doc.children)
        if (c->name == "scene") { sceneNode = c.get(); break; }
    if (!sceneNode) { SetLastError("no <scene> element in " + path); return false; }
    Graph graph;
    Value* root = nullptr;
    if (!graph.Build(*sceneNode, &root)) { SetLastError("failed to build value graph: " + graph.error); return false; }

    CScene& S = *scene;
    MaterialContext mc;
    mc.scenePath = path;
    mc.materials = &S.materials;
    mc.textureIndexBase = (uint32_t)S.textures.size();
    std::unordered_map<std::string, uint32_t> objToMesh;
    uint32_t rectangleMesh = kInvalidMaterialId;

    for (const auto& entry : root->nested) {
        const std::string& tag = entry.first;
        const Value& obj = *entry.second;
        if (KeywordIs(tag, "integrator")) {
            const std::string type = obj.GetString("type", "");
            if (KeywordIs(type, "path")) S.maxBounceCount = (uint32_t)obj.GetInt("max_depth", 3);
            else std::fprintf(stderr, "dcrt: unsupported integrator type '%s'\n", type.c_str());
        } else if (KeywordIs(tag, "sensor")) {
            const std::string type = obj.GetString("type", "");
            if (KeywordIs(type, "perspective")) S.cameraType = ECameraType::PinHole;
            else if (KeywordIs(type, "thinlens")) S.cameraType = ECameraType::ThinLens;
            else std::fprintf(stderr, "dcrt: unsupported sensor type '%s'\n", type.c_str());
            {
                Float3 position(0.0f, 0.0f, 0.0f), euler(0.0f, 0.0f, 0.0f);
                if (Value* t = obj.Field("to_world")) {
                    position = Float3(t->m.m[3][0], t->m.m[3][1], t->m.m[3][2]);
                    euler = MatrixRotationToRollPitchYaw(t->m);
                }
                S.camera.position = position;
                S.camera.eulerAngles = euler;
            }
            if (Value* film = obj.FirstNested("film")) {
                S.resolutionWidth = (uint32_t)film->GetInt("width", 768);
                S.resolutionHeight = (uint32_t)film->GetInt("height", 576);
                if (Value* rf = film->FirstNested("rfilter")) {
                    if (Value* tv = rf->Field("type")) {
                        const std::string& t = tv->s;
                        if (KeywordIs(t, "box")) {
                            S.filter = EFilter::Box;
                            S.filterRadius = rf->GetFloat("radius", 0.5f);
                        } else if (KeywordIs(t, "tent")) {
                            S.filter = EFilter::Triangle;
                            S.filterRadius = rf->GetFloat("radius", 1.0f);
                        } else if (KeywordIs(t, "gaussian")) {
                            S.filter = EFilter::Gaussian;
                            S.gaussianFilterAlpha = rf->GetFloat("stddev", 0.5f);
                            S.filterRadius = S.gaussianFilterAlpha * 4;
                        } else if (KeywordIs(t, "mitchell")) {
                            S.filter = EFilter::Mitchell;
                            S.mitchellB = rf->GetFloat("B", 1.0f / 3.0f);
                            S.mitchellB = rf->GetFloat("C", 1.0f / 3.0f);   // (quirk) C lands in B, :1169-1170
                            S.filterRadius = 2.0f;
                        } else if (KeywordIs(t, "lanczos")) {
                            S.filter = EFilter::LanczosSinc;
                            S.lanczosSincTau = (uint32_t)rf->GetInt("lobes", 3);
                            S.filterRadius = (float)S.lanczosSincTau;
                        } else {
                            std::fprintf(stderr, "dcrt: unsupported reconstruction filter '%s'\n", t.c_str());
                        }
                    }
                }
            }
            const float aspect = (float)S.resolutionWidth / (float)S.resolutionHeight;
            S.filmSize.x = 0.035f;                                   // (quirk) fixed 35 mm, :1191-1192
            S.filmSize.y = S.filmSize.x / std::fmax(aspect, 0.0001f);
            if (Value* fl = obj.Field("focal_length")) {
                S.focalLength = (float)std::atof(fl->s.c_str()) * 0.001f;   // "50mm" -> 0.05
                if (S.cameraType == ECameraType::PinHole) std::fprintf(stderr, "dcrt: focal length on a PinHole camera is not supported\n");
            } else {
                S.focalLength = 0.05f;
            }
            float fovDeg = 50.0f;
            if (Value* fv = obj.Field("fov")) {
                if (fv->type == VT::Float) {
                    fovDeg = std::clamp(fv->f, 0.0001f, 179.99f);
                    if (S.cameraType == ECameraType::ThinLens) std::fprintf(stderr, "dcrt: fov on a ThinLens camera is not supported\n");
                }
            }
            S.fovX = fovDeg * (kPi / 180.0f);                       // XMConvertToRadians
            if (S.cameraType == ECameraType::PinHole) {
                const std::string axis = obj.GetString("fov_axis", "x");
                if (KeywordIs(axis, "x")) {
                } else if (KeywordIs(axis, "y")) {
                    S.fovX *= aspect;
                } else {
                    std::fprintf(stderr, "dcrt: unsupported fov_axis '%s'\n", axis.c_str());
                }
            } else if (S.cameraType == ECameraType::ThinLens) {
                Value* ar = obj.Field("aperture_radius");
                S.relativeAperture = ar ? S.focalLength / (ar->UnionFloat() * 2) : 8.0f;
                Value* fd = obj.Field("focus_distance");
                S.focalDistance = fd ? fd->UnionFloat() : 2.0f;
            }
        } else if (KeywordIs(tag, "bsdf")) {
            uint32_t id = 0;
            mc.CreateAndAdd(obj, &id);
        } else if (KeywordIs(tag, "shape")) {
            Value* typeValue = obj.Field("type");
            if (!typeValue) { std::fprintf(stderr, "dcrt: cannot determine the type of shape\n"); continue; }
            Value* tw = obj.Field("to_world");
            const Float4x4 transform = tw ? tw->m : Float4x4::Identity();
            Value* emitter = obj.FirstNested("emitter");
            const bool isLight = emitter != nullptr;
            uint32_t materialId = kInvalidMaterialId;
            if (Value* b = obj.FirstNested("bsdf")) {
                auto it = mc.bsdfToId.find(b);
                if (it == mc.bsdfToId.end()) mc.CreateAndAdd(*b, &materialId);
                else materialId = it->second;
            } else if (isLight) {
                // a pitch-black non-reflective material for an emitter-only shape (:1282-1300)
                materialId = (uint32_t)S.materials.size();
                SMaterial lm;
                lm.albedo = Float3(0.0f, 0.0f, 0.0f);
                lm.roughness = 0.0f;
                lm.ior = Float3(1.0f, 1.0f, 1.0f);
                lm.opacity = 1.0f;
                lm.type = EMaterialType::Diffuse;
                lm.albedoTextureIndex = -1;
                lm.opacityTextureIndex = -1;
                lm.multiscattering = false;
                lm.isTwoSided = false;
                lm.hasRoughnessTexture = false;
                lm.internalScatteringMode = DCRT_INTERNAL_SCATTERING_MULTIPLE;
                lm.name = "LightMaterial";
                S.materials.push_back(lm);
            }
            bool created = false;
            uint32_t meshIndex = 0;
            const std::string& st = typeValue->s;
            if (st == "obj") {
                Value* fn = obj.Field("filename");
                if (!fn) {
                    std::fprintf(stderr, "dcrt: cannot find filename of an obj shape\n");
                } else {
                    const std::string file = mc.Absolute(fn->s);
                    auto it = objToMesh.find(file);
                    if (it != objToMesh.end()) {       // one mesh per file, instanced (:1326-1331)
                        meshIndex = it->second;
                        created = true;
                    } else {
                        ObjData data;
                        std::string err;
                        SMeshProcessingParams params;
                        params.applyTransform = false;
                        params.changeWindingOrder = true;
                        params.flipTexcoordV = true;
                        Mesh mesh;
                        if (ParseObjFile(file, &data, &err) &&
                            CreateMeshFromObjData(data, data.shapes.data(), (uint32_t)data.shapes.size(), params, &mesh)) {
                            mesh.name = fn->s;
                            meshIndex = (uint32_t)S.meshes.size();
                            S.meshes.push_back(std::move(mesh));
                            objToMesh.insert({ file, meshIndex });
                            created = true;
                        } else {
                            std::fprintf(stderr, "dcrt: failed to load wavefront obj file '%s' %s\n", file.c_str(), err.c_str());
                        }
                    }
                }
            } else if (st == "rectangle") {
                if (rectangleMesh == kInvalidMaterialId) {
                    // generated once with the first rectangle's material; later rectangles
                    // share it and take their material from the instance override (:1358-1378)
                    Mesh mesh;
                    if (!mesh.GenerateRectangle(materialId, true, Float4x4::Identity())) {
                        std::fprintf(stderr, "dcrt: failed to generate rectangle shape\n");
                        continue;
                    }
                    mesh.name = "rectangle";
                    rectangleMesh = (uint32_t)S.meshes.size();
                    S.meshes.push_back(std::move(mesh));
                }
                meshIndex = rectangleMesh;
                created = true;
            } else {
                std::fprintf(stderr, "dcrt: unsupported shape type '%s'\n", st.c_str());
            }
            if (!created) continue;
            std::string name;
            if (Value* idv = obj.Field("id")) name = idv->s;
            else {
                char buf[64];
                std::snprintf(buf, sizeof(buf), "Unnamed shape %03u", (uint32_t)S.meshInstances.size());
                name = buf;
            }
            const uint32_t instanceIndex = (uint32_t)S.meshInstances.size();
            SMeshInstance inst;
            inst.name = name;
            inst.meshIndex = meshIndex;
            inst.materialIdOverride = materialId;
            S.meshInstances.push_back(inst);
            S.instanceTransforms.push_back(Float4x3::From4x4(transform));
            if (S.GetLightCount() >= DCRT_MAX_LIGHT_COUNT) {
                std::fprintf(stderr, "dcrt: an emitter is discarded since the maximum light count is hit\n");
                continue;
            }
            if (isLight) {
                Value* et = emitter->Field("type");
                if (et && et->type == VT::String) {
                    if (KeywordIs(et->s, "area")) {
                        SMeshLight light;
                        light.instanceIndex = instanceIndex;
                        light.color = emitter->GetVec("radiance", Float3(1.0f, 1.0f, 1.0f));
                        S.meshLights.push_back(light);
                    } else {
                        std::fprintf(stderr, "dcrt: unsupported emitter type nested in a shape '%s'\n", et->s.c_str());
                    }
                } else {
                    std::fprintf(stderr, "dcrt: cannot determine emitter type\n");
                }
            }
        } else if (KeywordIs(tag, "emitter")) {
            Value* et = obj.Field("type");
            if (!et || et->type != VT::String) { std::fprintf(stderr, "dcrt: cannot determine emitter type\n"); continue; }
            if (S.GetLightCount() >= DCRT_MAX_LIGHT_COUNT) {
                std::fprintf(stderr, "dcrt: an emitter is discarded since the maximum light count is hit\n");
                continue;
            }
            if (KeywordIs(et->s, "constant")) {
                if (S.hasEnvironmentLight) {
                    std::fprintf(stderr, "dcrt: more than one constant emitter is not supported\n");
                    continue;
                }
                S.hasEnvironmentLight = true;
                S.environmentLight = SEnvironmentLight();
                S.environmentLight.color = obj.GetVec("radiance", Float3(1.0f, 1.0f, 1.0f));
            } else if (KeywordIs(et->s, "directional")) {
                SPunctualLight light;
                light.isDirectional = true;
                light.SetEulerAnglesFromDirection(Float3(0.0f, -1.0f, 0.0f));
                light.color = obj.GetVec("irradiance", Float3(1.0f, 1.0f, 1.0f));
                if (Value* dv = obj.Field("direction")) {
                    if (dv->type == VT::Vector) light.SetEulerAnglesFromDirection(dv->v);
                    else std::fprintf(stderr, "dcrt: non-vector direction type is not supported\n");
                }
                S.punctualLights.push_back(light);
            } else {
                std::fprintf(stderr, "dcrt: unsupported emitter type '%s'\n", et->s.c_str());
            }
        }
    }
    // textures in first-reference order (LoadTexturesFromFiles, :925-958)
    for (const auto& t : mc.textures) {
        CTexture tex;
        tex.name = t.second;
        if (!LoadTextureFile(t.first, &tex)) std::fprintf(stderr, "dcrt: loading texture from file \"%s\" failed\n", t.first.c_str());
        S.textures.push_back(std::move(tex));
    }
    return true;
}

}  // namespace dcrt
