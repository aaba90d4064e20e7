// scene_loader.cpp -- Nori XML scene format -> flattened nori_scene_desc.
//
// Host-side plugin boundary.  It keeps the reference's object model so an
// unchanged scene file selects this path:
//   * a NoriObject factory keyed by the XML `type` name (object.h:130-186);
//   * typed PropertyList accessors with the same names and defaults
//     (proplist.cpp:23-61; missing required property -> error);
//   * loadFromXML's tag table, transform composition and object lifecycle
//     ctor(props) -> addChild -> setParent -> activate (parser.cpp:28-338);
//   * WavefrontOBJ loading with quad split and vertex de-duplication
//     (obj.cpp:32-132).
// Plugins outside this path's scope (photonmapper, image textures, normal
// maps, Perlin noise) are rejected with NORI_ERR_UNSUPPORTED.
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <memory>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "host_scene.h"

namespace nori {

// ------------------------------------------------------------------ XML
struct XmlNode {
    std::string name;
    std::vector<std::pair<std::string, std::string>> attrs;
    std::vector<XmlNode> children;
    int line = 0;
    const std::string *attr(const std::string &k) const {
        for (auto &a : attrs)
            if (a.first == k) return &a.second;
        return nullptr;
    }
};

class XmlParser {
  public:
    XmlParser(const std::string &text, const std::string &file) : s_(text), file_(file) {}
    XmlNode parse() {
        skip_misc();
        if (pos_ >= s_.size() || s_[pos_] != '<') fail("expected root element");
        XmlNode root = element();
        skip_misc();
        if (pos_ < s_.size()) fail("unexpected content after root element");
        return root;
    }

  private:
    const std::string &s_;
    std::string file_;
    size_t pos_ = 0;
    int line_at(size_t p) const {
        int l = 1;
        for (size_t i = 0; i < p && i < s_.size(); ++i) l += s_[i] == '\n';
        return l;
    }
    [[noreturn]] void fail(const std::string &m) const {
        throw NoriException(NORI_ERR_PARSE, "Error while parsing \"" + file_ + "\": " + m + " (at row " +
                                                std::to_string(line_at(pos_)) + ")");
    }
    void skip_ws() {
        while (pos_ < s_.size() && std::isspace((unsigned char)s_[pos_])) ++pos_;
    }
    bool starts(const char *p) const { return s_.compare(pos_, std::strlen(p), p) == 0; }
    void skip_misc() {  // whitespace, comments, declarations, processing instructions
        for (;;) {
            skip_ws();
            if (starts("<!--")) {
                size_t e = s_.find("-->", pos_ + 4);
                if (e == std::string::npos) fail("unterminated comment");
                pos_ = e + 3;
            } else if (starts("<?")) {
                size_t e = s_.find("?>", pos_ + 2);
                if (e == std::string::npos) fail("unterminated declaration");
                pos_ = e + 2;
            } else if (starts("<!")) {
                size_t e = s_.find('>', pos_ + 2);
                if (e == std::string::npos) fail("unterminated doctype");
                pos_ = e + 1;
            } else {
                return;
            }
        }
    }
    std::string name_tok() {
        size_t b = pos_;
        while (pos_ < s_.size() && (std::isalnum((unsigned char)s_[pos_]) || s_[pos_] == '_' || s_[pos_] == '-' ||
                                    s_[pos_] == ':' || s_[pos_] == '.'))
            ++pos_;
        if (b == pos_) fail("expected a name");
        return s_.substr(b, pos_ - b);
    }
    static std::string unescape(const std::string &v) {
        std::string r;
        for (size_t i = 0; i < v.size(); ++i) {
            if (v[i] == '&') {
                size_t e = v.find(';', i);
                std::string ent = e == std::string::npos ? "" : v.substr(i + 1, e - i - 1);
                if (ent == "lt") r += '<';
                else if (ent == "gt") r += '>';
                else if (ent == "amp") r += '&';
                else if (ent == "quot") r += '"';
                else if (ent == "apos") r += '\'';
                else { r += v[i]; continue; }
                i = e;
            } else {
                r += v[i];
            }
        }
        return r;
    }
    XmlNode element() {
        XmlNode n;
        n.line = line_at(pos_);
        ++pos_;  // '<'
        n.name = name_tok();
        for (;;) {
            skip_ws();
            if (pos_ >= s_.size()) fail("unterminated tag");
            if (s_[pos_] == '/') {
                if (pos_ + 1 >= s_.size() || s_[pos_ + 1] != '>') fail("malformed tag end");
                pos_ += 2;
                return n;
            }
            if (s_[pos_] == '>') {
                ++pos_;
                break;
            }
            std::string k = name_tok();
            skip_ws();
            if (pos_ >= s_.size() || s_[pos_] != '=') fail("expected '=' after attribute");
            ++pos_;
            skip_ws();
            char q = pos_ < s_.size() ? s_[pos_] : 0;
            if (q != '"' && q != '\'') fail("expected quoted attribute value");
            size_t e = s_.find(q, pos_ + 1);
            if (e == std::string::npos) fail("unterminated attribute value");
            n.attrs.emplace_back(k, unescape(s_.substr(pos_ + 1, e - pos_ - 1)));
            pos_ = e + 1;
        }
        for (;;) {  // content
            skip_misc();
            if (pos_ >= s_.size()) fail("unterminated element <" + n.name + ">");
            if (starts("</")) {
                pos_ += 2;
                std::string nm = name_tok();
                if (nm != n.name) fail("mismatched closing tag </" + nm + "> for <" + n.name + ">");
                skip_ws();
                if (pos_ >= s_.size() || s_[pos_] != '>') fail("malformed closing tag");
                ++pos_;
                return n;
            }
            if (s_[pos_] == '<') {
                n.children.push_back(element());
            } else {
                fail("unexpected content");  // parser.cpp:133-136: text is an error
            }
        }
    }
};

// ------------------------------------------------------------------ helpers
static std::vector<std::string> tokenize(const std::string &s, const std::string &delim = ", ") {
    std::vector<std::string> t;  // common.cpp:147-163 (includeEmpty = false)
    size_t last = 0, pos = s.find_first_of(delim, last);
    while (last != std::string::npos) {
        if (pos != last) t.push_back(s.substr(last, pos - last));
        last = pos;
        if (last != std::string::npos) {
            last += 1;
            pos = s.find_first_of(delim, last);
        }
    }
    return t;
}
static float to_float(const std::string &s) {  // common.cpp:103-109
    char *end = nullptr;
    float r = std::strtof(s.c_str(), &end);
    if (*end != '\0') throw NoriException(NORI_ERR_PARSE, "Could not parse floating point value \"" + s + "\"");
    return r;
}
static int to_int(const std::string &s) {
    char *end = nullptr;
    int r = (int)std::strtol(s.c_str(), &end, 10);
    if (*end != '\0') throw NoriException(NORI_ERR_PARSE, "Could not parse integer value \"" + s + "\"");
    return r;
}
static unsigned to_uint(const std::string &s) {
    char *end = nullptr;
    unsigned r = (unsigned)std::strtoul(s.c_str(), &end, 10);
    if (*end != '\0') throw NoriException(NORI_ERR_PARSE, "Could not parse integer value \"" + s + "\"");
    return r;
}
static bool to_bool(const std::string &s) {
    std::string v;
    for (char c : s) v += (char)std::tolower((unsigned char)c);
    if (v == "true") return true;
    if (v == "false") return false;
    throw NoriException(NORI_ERR_PARSE, "Could not parse boolean value \"" + s + "\"");
}
static Vec3f to_vec3(const std::string &s) {
    auto t = tokenize(s);
    if (t.size() != 3) throw NoriException(NORI_ERR_PARSE, "Expected 3 values");
    return Vec3f{to_float(t[0]), to_float(t[1]), to_float(t[2])};
}

// 4x4 float matrices, row-major; product in Eigen's k-order.
Mat4 mat_identity() {
    Mat4 m{};
    for (int i = 0; i < 4; ++i) m.m[4 * i + i] = 1.0f;
    return m;
}
Mat4 mat_mul(const Mat4 &a, const Mat4 &b) {
    Mat4 r{};
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j)
            r.m[4 * i + j] = ((a.m[4 * i + 0] * b.m[0 + j] + a.m[4 * i + 1] * b.m[4 + j]) + a.m[4 * i + 2] * b.m[8 + j]) +
                             a.m[4 * i + 3] * b.m[12 + j];
    return r;
}
bool mat_inverse(const Mat4 &a, Mat4 &out) {  // Gauss-Jordan in double, rounded once
    double m[4][8];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 8; ++j) m[i][j] = j < 4 ? a.m[4 * i + j] : (j - 4 == i ? 1.0 : 0.0);
    for (int c = 0; c < 4; ++c) {
        int p = c;
        for (int r = c + 1; r < 4; ++r)
            if (std::fabs(m[r][c]) > std::fabs(m[p][c])) p = r;
        if (m[p][c] == 0.0) return false;
        if (p != c)
            for (int j = 0; j < 8; ++j) std::swap(m[p][j], m[c][j]);
        double iv = 1.0 / m[c][c];
        for (int j = 0; j < 8; ++j) m[c][j] *= iv;
        for (int r = 0; r < 4; ++r) {
            if (r == c) continue;
            double f = m[r][c];
            for (int j = 0; j < 8; ++j) m[r][j] -= f * m[c][j];
        }
    }
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) out.m[4 * i + j] = (float)m[i][j + 4];
    return true;
}
static Vec3f xf_point(const Mat4 &t, Vec3f p) {  // transform.h:81-84
    float r[4];
    for (int i = 0; i < 4; ++i)
        r[i] = ((t.m[4 * i] * p.x + t.m[4 * i + 1] * p.y) + t.m[4 * i + 2] * p.z) + t.m[4 * i + 3] * 1.0f;
    return Vec3f{r[0] / r[3], r[1] / r[3], r[2] / r[3]};
}
static Vec3f normalized(Vec3f v) {
    float n = std::sqrt((v.x * v.x + v.y * v.y) + v.z * v.z);
    return Vec3f{v.x / n, v.y / n, v.z / n};
}
static Vec3f vcross(Vec3f a, Vec3f b) {
    return Vec3f{a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x};
}

// ------------------------------------------------------------------ PropertyList
struct Property {
    enum Type { Bool, Int, Float, String, Color, Point3, Vector3, Point2, Vector2, Transform } type;
    bool b = false;
    int i = 0;
    float f = 0;
    std::string s;
    Vec3f v{};
    float v2[2] = {0, 0};
    Mat4 t{};
};
static const char *type_name(Property::Type t) {
    static const char *n[] = {"boolean", "integer", "float", "string", "color", "point", "vector", "point", "vector", "transform"};
    return n[t];
}
class PropertyList {  // proplist.cpp:23-61
  public:
    void set(const std::string &name, const Property &p) {
        if (props_.count(name)) std::fprintf(stderr, "Property \"%s\" was specified multiple times!\n", name.c_str());
        props_[name] = p;
    }
    bool has(const std::string &n) const { return props_.count(n) != 0; }
    const Property *get(const std::string &n, Property::Type t) const {
        auto it = props_.find(n);
        if (it == props_.end()) return nullptr;
        if (it->second.type != t)
            throw NoriException(NORI_ERR_PARSE, "Property '" + n + "' has the wrong type! (expected <" +
                                                    type_name(t) + ">)!");
        return &it->second;
    }
    const Property &req(const std::string &n, Property::Type t) const {
        const Property *p = get(n, t);
        if (!p) throw NoriException(NORI_ERR_PARSE, "Property '" + n + "' is missing!");
        return *p;
    }
    bool getBoolean(const std::string &n, bool d) const { auto p = get(n, Property::Bool); return p ? p->b : d; }
    int getInteger(const std::string &n, int d) const { auto p = get(n, Property::Int); return p ? p->i : d; }
    float getFloat(const std::string &n, float d) const { auto p = get(n, Property::Float); return p ? p->f : d; }
    float getFloat(const std::string &n) const { return req(n, Property::Float).f; }
    std::string getString(const std::string &n, const std::string &d) const { auto p = get(n, Property::String); return p ? p->s : d; }
    std::string getString(const std::string &n) const { return req(n, Property::String).s; }
    Vec3f getColor(const std::string &n, Vec3f d) const { auto p = get(n, Property::Color); return p ? p->v : d; }
    Vec3f getColor(const std::string &n) const { return req(n, Property::Color).v; }
    Vec3f getPoint3(const std::string &n, Vec3f d) const { auto p = get(n, Property::Point3); return p ? p->v : d; }
    Vec3f getVector3(const std::string &n, Vec3f d) const { auto p = get(n, Property::Vector3); return p ? p->v : d; }
    Vec3f getVector3(const std::string &n) const { return req(n, Property::Vector3).v; }
    Vec3f getPoint3(const std::string &n) const { return req(n, Property::Point3).v; }
    void getPoint2(const std::string &n, float out[2], float d0, float d1) const {
        auto p = get(n, Property::Point2);
        out[0] = p ? p->v2[0] : d0;
        out[1] = p ? p->v2[1] : d1;
    }
    void getVector2(const std::string &n, float out[2], float d0, float d1) const {
        auto p = get(n, Property::Vector2);
        out[0] = p ? p->v2[0] : d0;
        out[1] = p ? p->v2[1] : d1;
    }
    Mat4 getTransform(const std::string &n, const Mat4 &d) const { auto p = get(n, Property::Transform); return p ? p->t : d; }

  private:
    std::map<std::string, Property> props_;
};

// ------------------------------------------------------------------ NoriObject
enum EClassType {  // object.h:34-48
    EScene = 0, EMesh, ETexture, EBSDF, EPhaseFunction, EEmitter, EMedium, ECamera, EIntegrator, ESampler, ETest,
    EReconstructionFilter, EClassTypeCount
};
static const char *class_name(int t) {
    static const char *n[] = {"scene", "mesh", "texture", "bsdf", "phase", "emitter", "medium", "camera",
                              "integrator", "sampler", "test", "rfilter"};
    return t >= 0 && t < EClassTypeCount ? n[t] : "unknown";
}

struct NoriObject {
    virtual ~NoriObject() = default;
    virtual EClassType getClassType() const = 0;
    virtual void addChild(NoriObject *child) {
        throw NoriException(NORI_ERR_PARSE, std::string("NoriObject::addChild() is not implemented for objects of type '") +
                                                class_name(getClassType()) + "'!");
    }
    virtual void setParent(NoriObject *) {}
    virtual void activate() {}
    std::string idName;
};
using Ctor = std::function<NoriObject *(const PropertyList &)>;
static std::map<std::string, Ctor> &registry() {
    static std::map<std::string, Ctor> r;
    return r;
}
struct Registrar {
    Registrar(const char *name, Ctor c) { registry()[name] = std::move(c); }
};
#define NORI_REGISTER_CLASS(cls, name) \
    static Registrar cls##_reg_(name, [](const PropertyList &p) -> NoriObject * { return new cls(p); });

// Out-of-scope plugins: recognised so the error says why.
struct Unsupported : NoriObject {
    EClassType getClassType() const override { return EClassTypeCount; }
};
static const char *kUnsupported[] = {"checkerboard_float", "perlin", "chi2test"};

// ---- textures (consttexture.cpp)
struct ConstantColor : NoriObject {
    Vec3f value;
    explicit ConstantColor(const PropertyList &p) : value(p.getColor("value", Vec3f{0, 0, 0})) {}
    EClassType getClassType() const override { return ETexture; }
};
NORI_REGISTER_CLASS(ConstantColor, "constant_color")
struct ConstantFloat : NoriObject {
    float value;
    explicit ConstantFloat(const PropertyList &p) : value(p.getFloat("value", 0.f)) {}
    EClassType getClassType() const override { return ETexture; }
};
NORI_REGISTER_CLASS(ConstantFloat, "constant_float")
struct CheckerboardColor : NoriObject {  // checkerboard.cpp:62-68 (Checkerboard<Color3f>)
    Vec3f value1, value2;
    float delta[2], scale[2];
    explicit CheckerboardColor(const PropertyList &p)
        : value1(p.getColor("value1", Vec3f{0, 0, 0})), value2(p.getColor("value2", Vec3f{1, 1, 1})) {
        p.getPoint2("delta", delta, 0.f, 0.f);
        p.getVector2("scale", scale, 1.f, 1.f);
    }
    EClassType getClassType() const override { return ETexture; }
};
NORI_REGISTER_CLASS(CheckerboardColor, "checkerboard_color")
// ImageTexture (imagetexture.cpp:69-85) and NormalMap (normalmap.cpp:69-85):
// "fileName" (default textures/default.png, resolved against the scene's
// directory) decoded at construction like stbi_load(.., STBI_rgb), "wrap"
// repeat | clamp (common.h:274-283).  Evaluated on the device (albedo_at,
// surface) and by the oracle.
struct ImageTex : NoriObject {
    bool normal_map;
    int width = 0, height = 0, wrap = NORI_WRAP_REPEAT;
    std::vector<uint8_t> rgb;
    ImageTex(const PropertyList &p, bool nm) : normal_map(nm) {
        const std::string file = p.getString("fileName", "textures/default.png");
        const std::string w = p.getString("wrap", "repeat");
        if (w == "repeat") wrap = NORI_WRAP_REPEAT;
        else if (w == "clamp") wrap = NORI_WRAP_CLAMP;
        else throw NoriException(NORI_ERR_PARSE, "Invalid wrap type name " + w);
        if (file.empty()) throw NoriException(NORI_ERR_PARSE, "No image data was loaded!");
        decode_image_rgb8(resolve_path(file), width, height, rgb);
    }
    EClassType getClassType() const override { return ETexture; }
};
struct ImageTexture : ImageTex {
    explicit ImageTexture(const PropertyList &p) : ImageTex(p, false) {}
};
NORI_REGISTER_CLASS(ImageTexture, "ImageTexture")
struct NormalMap : ImageTex {
    explicit NormalMap(const PropertyList &p) : ImageTex(p, true) {}
};
NORI_REGISTER_CLASS(NormalMap, "NormalMap")

// ---- BSDFs
struct Bsdf : NoriObject {
    nori_bsdf_desc d{};
    const ImageTex *image = nullptr;  // diffuse ImageTexture albedo
    // consumed children (textures) stay alive until the BSDF dies: the parser
    // calls setParent on a child after addChild (parser.cpp:208-211)
    std::vector<std::unique_ptr<NoriObject>> consumed;
    EClassType getClassType() const override { return EBSDF; }
};
struct Diffuse : Bsdf {  // diffuse.cpp:29-66
    bool has_albedo = false;
    explicit Diffuse(const PropertyList &p) {
        d.type = NORI_BSDF_DIFFUSE;
        if (p.has("albedo")) {
            Vec3f a = p.getColor("albedo");
            d.albedo[0] = a.x; d.albedo[1] = a.y; d.albedo[2] = a.z;
            has_albedo = true;
        }
    }
    void addChild(NoriObject *o) override {
        if (o->getClassType() != ETexture)
            throw NoriException(NORI_ERR_PARSE, std::string("Diffuse::addChild(<") + class_name(o->getClassType()) + ">) is not supported!");
        if (o->idName != "albedo") throw NoriException(NORI_ERR_PARSE, "The name of this texture does not match any field!");
        if (has_albedo) throw NoriException(NORI_ERR_PARSE, "There is already an albedo defined!");
        if (auto *c = dynamic_cast<ConstantColor *>(o)) {
            d.albedo[0] = c->value.x; d.albedo[1] = c->value.y; d.albedo[2] = c->value.z;
        } else if (auto *t = dynamic_cast<ImageTex *>(o)) {
            d.albedo_texture = NORI_TEXTURE_IMAGE;  // (a NormalMap named "albedo" evaluates its own way)
            if (t->normal_map) throw NoriException(NORI_ERR_UNSUPPORTED, "a NormalMap as a diffuse albedo");
            image = t;
        } else if (auto *k = dynamic_cast<CheckerboardColor *>(o)) {
            d.albedo_texture = NORI_TEXTURE_CHECKERBOARD;
            d.albedo[0] = k->value1.x; d.albedo[1] = k->value1.y; d.albedo[2] = k->value1.z;
            d.tex_value2[0] = k->value2.x; d.tex_value2[1] = k->value2.y; d.tex_value2[2] = k->value2.z;
            d.tex_delta[0] = k->delta[0]; d.tex_delta[1] = k->delta[1];
            d.tex_scale[0] = k->scale[0]; d.tex_scale[1] = k->scale[1];
        } else {
            throw NoriException(NORI_ERR_UNSUPPORTED, "albedo textures: constant_color, checkerboard_color and ImageTexture are on this path");
        }
        has_albedo = true;
        consumed.emplace_back(o);
    }
    void activate() override {
        if (!has_albedo) { d.albedo[0] = d.albedo[1] = d.albedo[2] = 0.5f; has_albedo = true; }
    }
};
NORI_REGISTER_CLASS(Diffuse, "diffuse")
struct Mirror : Bsdf {
    explicit Mirror(const PropertyList &) { d.type = NORI_BSDF_MIRROR; }
};
NORI_REGISTER_CLASS(Mirror, "mirror")
struct Dielectric : Bsdf {  // dielectric.cpp:26-31
    explicit Dielectric(const PropertyList &p) {
        d.type = NORI_BSDF_DIELECTRIC;
        d.int_ior = p.getFloat("intIOR", 1.5046f);
        d.ext_ior = p.getFloat("extIOR", 1.000277f);
    }
};
NORI_REGISTER_CLASS(Dielectric, "dielectric")
struct Microfacet : Bsdf {  // microfacet.cpp:26-45
    explicit Microfacet(const PropertyList &p) {
        d.type = NORI_BSDF_MICROFACET;
        d.alpha = p.getFloat("alpha", 0.1f);
        d.int_ior = p.getFloat("intIOR", 1.5046f);
        d.ext_ior = p.getFloat("extIOR", 1.000277f);
        Vec3f kd = p.getColor("kd", Vec3f{0.5f, 0.5f, 0.5f});
        d.kd[0] = kd.x; d.kd[1] = kd.y; d.kd[2] = kd.z;
    }
};
NORI_REGISTER_CLASS(Microfacet, "microfacet")
struct Disney : Bsdf {  // disney.cpp:46-60
    explicit Disney(const PropertyList &p) {
        d.type = NORI_BSDF_DISNEY;
        d.metallic = p.getFloat("metallic", 0.0f);
        d.specular = p.getFloat("specular", 0.0f);
        d.roughness = p.getFloat("roughness", 0.0f);
        d.sheen = p.getFloat("sheen", 0.0f);
        d.sheen_tint = p.getFloat("sheenTint", 0.0f);
        d.specular_tint = p.getFloat("specularTint", 0.0f);
        Vec3f b = p.getColor("baseColor", Vec3f{0, 0, 0});
        d.base_color[0] = b.x; d.base_color[1] = b.y; d.base_color[2] = b.z;
    }
    void addChild(NoriObject *o) override { consumed.emplace_back(o); }  // disney.cpp:176: ignores children
};
NORI_REGISTER_CLASS(Disney, "disney")

// ---- emitters
struct Emitter : NoriObject {
    nori_emitter_desc d{};
    std::vector<float> rgb;
    EClassType getClassType() const override { return EEmitter; }
};
struct AreaEmitter : Emitter {  // arealight.cpp:25-28
    explicit AreaEmitter(const PropertyList &p) {
        d.type = NORI_EMITTER_AREA;
        Vec3f r = p.getColor("radiance");
        d.radiance[0] = r.x; d.radiance[1] = r.y; d.radiance[2] = r.z;
        d.shape = -1;
    }
};
NORI_REGISTER_CLASS(AreaEmitter, "area")
struct EnvMapEmitter : Emitter {  // envmap.cpp:13-58
    explicit EnvMapEmitter(const PropertyList &p) {
        d.type = NORI_EMITTER_ENVMAP;
        d.shape = -1;
        d.weight = p.getFloat("weight", 1.0f);
        std::string fn = resolve_path(p.getString("filename", "textures/envmaptext.exr"));
        Vec3f ls = p.getVector3("luminanceScale", Vec3f{0.3f, 0.6f, 0.1f});
        d.lum_scale[0] = ls.x;
        d.lum_scale[1] = ls.y;
        d.lum_scale[2] = ls.z;
        int w = 0, h = 0;
        load_exr(fn, w, h, rgb);
        d.env_rows = h;  // Bitmap rows = scanlines (the envmap's "m_width")
        d.env_cols = w;
        if (h < 2 || w < 2) throw NoriException(NORI_ERR_INVALID, "EnvMap: the image needs at least 2x2 texels");
    }
};
NORI_REGISTER_CLASS(EnvMapEmitter, "envmap")
struct PointEmitter : Emitter {  // pointlight.cpp:11-15
    explicit PointEmitter(const PropertyList &p) {
        d.type = NORI_EMITTER_POINT;
        d.shape = -1;
        Vec3f q = p.getPoint3("position", Vec3f{0, 0, 0}), w = p.getColor("power", Vec3f{0, 0, 0});
        d.position[0] = q.x; d.position[1] = q.y; d.position[2] = q.z;
        d.power[0] = w.x; d.power[1] = w.y; d.power[2] = w.z;
    }
};
NORI_REGISTER_CLASS(PointEmitter, "point")
struct SpotEmitter : Emitter {  // spotlight.cpp:11-18
    explicit SpotEmitter(const PropertyList &p) {
        d.type = NORI_EMITTER_SPOT;
        d.shape = -1;
        Vec3f q = p.getPoint3("position"), c = p.getColor("color"), dir = normalized(p.getVector3("direction"));
        d.position[0] = q.x; d.position[1] = q.y; d.position[2] = q.z;
        d.power[0] = c.x; d.power[1] = c.y; d.power[2] = c.z;
        d.direction[0] = dir.x; d.direction[1] = dir.y; d.direction[2] = dir.z;
        // std::cos(M_PI / 180 * deg): M_PI is a float literal (common.h:56), the cos is the float overload
        d.cos_falloff_start = std::cos(3.14159265358979323846f / 180 * p.getFloat("falloffStart"));
        d.cos_total_width = std::cos(3.14159265358979323846f / 180 * p.getFloat("totalWidth"));
    }
};
NORI_REGISTER_CLASS(SpotEmitter, "spotlight")

// ---- shapes
struct Shape : NoriObject {
    NoriObject *bsdf = nullptr;
    Emitter *emitter = nullptr;
    ImageTex *normal_map = nullptr;
    std::vector<std::unique_ptr<NoriObject>> textures;  // textures added as children stay alive with the shape
    EClassType getClassType() const override { return EMesh; }
    ~Shape() override { delete bsdf; }
    void addChild(NoriObject *o) override {  // shape.cpp:42-74
        switch (o->getClassType()) {
        case EBSDF:
            if (bsdf) throw NoriException(NORI_ERR_PARSE, "Shape: tried to register multiple BSDF instances!");
            bsdf = o;
            break;
        case EEmitter:
            if (emitter) throw NoriException(NORI_ERR_PARSE, "Shape: tried to register multiple Emitter instances!");
            emitter = static_cast<Emitter *>(o);
            break;
        case ETexture:  // shape.cpp:59-67: a texture named "normal" is the normal map, others are ignored
            if (o->idName == "normal") {
                if (normal_map) throw NoriException(NORI_ERR_PARSE, "Shape: tried to register multiple Normal map instances!");
                auto *t = dynamic_cast<ImageTex *>(o);
                if (!t || !t->normal_map) throw NoriException(NORI_ERR_UNSUPPORTED, "normal maps: NormalMap textures only");
                normal_map = t;
            }
            textures.emplace_back(o);
            break;
        default:
            throw NoriException(NORI_ERR_PARSE, std::string("Shape::addChild(<") + class_name(o->getClassType()) + ">) is not supported!");
        }
    }
    void activate() override {  // shape.cpp:33-40: default diffuse BSDF
        if (!bsdf) {
            bsdf = registry().at("diffuse")(PropertyList());
            bsdf->activate();
        }
    }
};

struct Sphere : Shape {  // sphere.cpp:29-35
    Vec3f center;
    float radius;
    explicit Sphere(const PropertyList &p) {
        center = p.getPoint3("center", Vec3f{0, 0, 0});
        radius = p.getFloat("radius", 1.f);
    }
};
NORI_REGISTER_CLASS(Sphere, "sphere")

struct WavefrontOBJ : Shape {  // obj.cpp:32-132
    std::vector<float> V, N, UV;   // 3*n, 3*n, 2*n
    std::vector<uint32_t> F;       // 3*f (mesh-local)
    std::string name;
    explicit WavefrontOBJ(const PropertyList &p) {
        std::string fn = resolve_path(p.getString("filename"));
        std::ifstream is(fn);
        if (is.fail()) throw NoriException(NORI_ERR_IO, "Unable to open OBJ file \"" + fn + "\"!");
        Mat4 trafo = p.getTransform("toWorld", mat_identity());
        Mat4 inv;
        if (!mat_inverse(trafo, inv)) throw NoriException(NORI_ERR_PARSE, "singular toWorld transform");
        struct Key {
            uint32_t p = (uint32_t)-1, n = (uint32_t)-1, uv = (uint32_t)-1;
            bool operator==(const Key &o) const { return p == o.p && n == o.n && uv == o.uv; }
        };
        struct KeyHash {
            size_t operator()(const Key &v) const {
                size_t h = std::hash<uint32_t>()(v.p);
                h = h * 37 + std::hash<uint32_t>()(v.uv);
                h = h * 37 + std::hash<uint32_t>()(v.n);
                return h;
            }
        };
        std::vector<Vec3f> positions, normals;
        std::vector<std::pair<float, float>> texcoords;
        std::vector<Key> verts;
        std::vector<uint32_t> indices;
        std::unordered_map<Key, uint32_t, KeyHash> vmap;
        auto parse_vertex = [](const std::string &s) {
            auto t = tokenize_keep_empty(s, "/");
            if (t.size() < 1 || t.size() > 3) throw NoriException(NORI_ERR_PARSE, "Invalid vertex data: \"" + s + "\"");
            Key k;
            k.p = to_uint(t[0]);
            if (t.size() >= 2 && !t[1].empty()) k.uv = to_uint(t[1]);
            if (t.size() >= 3 && !t[2].empty()) k.n = to_uint(t[2]);
            return k;
        };
        std::string line;
        while (std::getline(is, line)) {
            std::istringstream ls(line);
            std::string prefix;
            ls >> prefix;
            if (prefix == "v") {
                Vec3f q{};
                ls >> q.x >> q.y >> q.z;
                positions.push_back(xf_point(trafo, q));
            } else if (prefix == "vt") {
                float u = 0, v = 0;
                ls >> u >> v;
                texcoords.emplace_back(u, v);
            } else if (prefix == "vn") {
                Vec3f n{};
                ls >> n.x >> n.y >> n.z;
                // transform.h:76-78: inverse-transpose, then normalized (obj.cpp:70)
                Vec3f r{(inv.m[0] * n.x + inv.m[4] * n.y) + inv.m[8] * n.z,
                        (inv.m[1] * n.x + inv.m[5] * n.y) + inv.m[9] * n.z,
                        (inv.m[2] * n.x + inv.m[6] * n.y) + inv.m[10] * n.z};
                normals.push_back(normalized(r));
            } else if (prefix == "f") {
                std::string a, b, c, d;
                ls >> a >> b >> c >> d;
                Key vs[6];
                int nv = 3;
                vs[0] = parse_vertex(a); vs[1] = parse_vertex(b); vs[2] = parse_vertex(c);
                if (!d.empty()) { vs[3] = parse_vertex(d); vs[4] = vs[0]; vs[5] = vs[2]; nv = 6; }
                for (int i = 0; i < nv; ++i) {
                    auto it = vmap.find(vs[i]);
                    if (it == vmap.end()) {
                        vmap[vs[i]] = (uint32_t)verts.size();
                        indices.push_back((uint32_t)verts.size());
                        verts.push_back(vs[i]);
                    } else {
                        indices.push_back(it->second);
                    }
                }
            }
        }
        F = std::move(indices);
        V.resize(3 * verts.size());
        for (size_t i = 0; i < verts.size(); ++i) {
            if (verts[i].p == 0 || verts[i].p > positions.size()) throw NoriException(NORI_ERR_PARSE, "OBJ: vertex index out of range in " + fn);
            Vec3f q = positions[verts[i].p - 1];
            V[3 * i] = q.x; V[3 * i + 1] = q.y; V[3 * i + 2] = q.z;
        }
        if (!normals.empty()) {
            N.resize(3 * verts.size());
            for (size_t i = 0; i < verts.size(); ++i) {
                if (verts[i].n == 0 || verts[i].n > normals.size()) throw NoriException(NORI_ERR_PARSE, "OBJ: normal index out of range in " + fn);
                Vec3f q = normals[verts[i].n - 1];
                N[3 * i] = q.x; N[3 * i + 1] = q.y; N[3 * i + 2] = q.z;
            }
        }
        if (!texcoords.empty()) {
            UV.resize(2 * verts.size());
            for (size_t i = 0; i < verts.size(); ++i) {
                if (verts[i].uv == 0 || verts[i].uv > texcoords.size()) throw NoriException(NORI_ERR_PARSE, "OBJ: uv index out of range in " + fn);
                UV[2 * i] = texcoords[verts[i].uv - 1].first; UV[2 * i + 1] = texcoords[verts[i].uv - 1].second;
            }
        }
        name = fn;
    }
    static std::vector<std::string> tokenize_keep_empty(const std::string &s, const std::string &delim) {
        std::vector<std::string> t;
        size_t last = 0, pos = s.find_first_of(delim, last);
        while (last != std::string::npos) {
            t.push_back(s.substr(last, pos == std::string::npos ? std::string::npos : pos - last));
            last = pos;
            if (last != std::string::npos) { last += 1; pos = s.find_first_of(delim, last); }
        }
        return t;
    }
};
NORI_REGISTER_CLASS(WavefrontOBJ, "obj")

// ---- reconstruction filters (rfilter.cpp)
struct RFilter : NoriObject {
    int type; float radius, p0 = 0, p1 = 0;
    EClassType getClassType() const override { return EReconstructionFilter; }
};
struct Gaussian : RFilter {
    explicit Gaussian(const PropertyList &p) { type = NORI_FILTER_GAUSSIAN; radius = p.getFloat("radius", 2.0f); p0 = p.getFloat("stddev", 0.5f); }
};
NORI_REGISTER_CLASS(Gaussian, "gaussian")
struct Mitchell : RFilter {
    explicit Mitchell(const PropertyList &p) { type = NORI_FILTER_MITCHELL; radius = p.getFloat("radius", 2.0f); p0 = p.getFloat("B", 1.0f / 3.0f); p1 = p.getFloat("C", 1.0f / 3.0f); }
};
NORI_REGISTER_CLASS(Mitchell, "mitchell")
struct Tent : RFilter {
    explicit Tent(const PropertyList &) { type = NORI_FILTER_TENT; radius = 1.0f; }
};
NORI_REGISTER_CLASS(Tent, "tent")
struct Box : RFilter {
    explicit Box(const PropertyList &) { type = NORI_FILTER_BOX; radius = 0.5f; }
};
NORI_REGISTER_CLASS(Box, "box")
struct Windowed : RFilter {
    explicit Windowed(const PropertyList &p) { type = NORI_FILTER_WINDOWED; radius = p.getFloat("radius", 2.0f); p0 = p.getFloat("tau", 1.0f); }
};
NORI_REGISTER_CLASS(Windowed, "windowed")

// ---- camera (perspective.cpp)
struct Perspective : NoriObject {
    nori_camera_desc d{};
    RFilter *filter = nullptr;
    explicit Perspective(const PropertyList &p, int type = NORI_CAMERA_PERSPECTIVE) {
        d.camera_type = type;
        d.width = p.getInteger("width", 1280);
        d.height = p.getInteger("height", 720);
        Mat4 c2w = p.getTransform("toWorld", mat_identity());
        std::memcpy(d.camera_to_world, c2w.m, sizeof(c2w.m));
        d.fov = p.getFloat("fov", 30.0f);
        d.near_clip = p.getFloat("nearClip", 1e-4f);
        d.far_clip = p.getFloat("farClip", 1e4f);
    }
    ~Perspective() override { delete filter; }
    EClassType getClassType() const override { return ECamera; }
    void addChild(NoriObject *o) override {
        if (o->getClassType() != EReconstructionFilter)
            throw NoriException(NORI_ERR_PARSE, std::string("Camera::addChild(<") + class_name(o->getClassType()) + ">) is not supported!");
        if (filter) throw NoriException(NORI_ERR_PARSE, "Camera: tried to register multiple reconstruction filters!");
        filter = static_cast<RFilter *>(o);
    }
    void activate() override {
        if (!filter) {
            filter = static_cast<RFilter *>(registry().at("gaussian")(PropertyList()));
            filter->activate();
        }
    }
};
NORI_REGISTER_CLASS(Perspective, "perspective")
struct ThinLens : Perspective {  // thinlens.cpp:30-51
    explicit ThinLens(const PropertyList &p) : Perspective(p, NORI_CAMERA_THINLENS) {
        d.focal_distance = p.getFloat("focalDist", 1.0f);
        d.lens_radius = p.getFloat("lensRadius", 0.0f);
    }
};
NORI_REGISTER_CLASS(ThinLens, "thinlens")
struct AdvancedCam : Perspective {  // advancedCamera.cpp:30-55
    explicit AdvancedCam(const PropertyList &p) : Perspective(p, NORI_CAMERA_ADVANCED) {
        d.focal_distance = p.getFloat("focalDist", 1.0f);
        d.lens_radius = p.getFloat("lensRadius", 0.0f);
        p.getVector2("distortion", d.distortion, 0.f, 0.f);
        Vec3f c = p.getVector3("chromaticAberation", Vec3f{0, 0, 0});
        d.chromatic[0] = c.x; d.chromatic[1] = c.y; d.chromatic[2] = c.z;
    }
};
NORI_REGISTER_CLASS(AdvancedCam, "advancedCamera")

// perspective.cpp:53-82, evaluated for the (possibly overridden) output size.
void compute_sample_to_camera(nori_camera_desc &d) {
    float aspect = d.width / (float)d.height;
    float recip = 1.0f / (d.far_clip - d.near_clip);
    float cot = 1.0f / std::tan((d.fov / 2.0f) * (3.14159265358979323846f / 180.0f));
    Mat4 P{};
    P.m[0] = cot; P.m[5] = cot;
    P.m[10] = d.far_clip * recip; P.m[11] = -d.near_clip * d.far_clip * recip;
    P.m[14] = 1.0f;
    Mat4 ST = mat_identity();  // Diagonal(0.5, -0.5*aspect, 1) * Translation(1, -1/aspect, 0)
    float sy = -0.5f * aspect;
    ST.m[0] = 0.5f; ST.m[5] = sy; ST.m[10] = 1.0f;
    ST.m[3] = 0.5f * 1.0f; ST.m[7] = sy * (-1.0f / aspect); ST.m[11] = 1.0f * 0.0f;
    Mat4 M = mat_mul(ST, P), inv;
    if (!mat_inverse(M, inv)) throw NoriException(NORI_ERR_PARSE, "degenerate camera projection");
    std::memcpy(d.sample_to_camera, inv.m, sizeof(inv.m));
}

// ---- sampler, integrators, medium, phase
struct Independent : NoriObject {  // independent.cpp:33-35
    int sampleCount;
    explicit Independent(const PropertyList &p) : sampleCount(p.getInteger("sampleCount", 1)) {}
    EClassType getClassType() const override { return ESampler; }
};
NORI_REGISTER_CLASS(Independent, "independent")
struct Integrator : NoriObject {
    int kind;
    explicit Integrator(int k) : kind(k) {}
    EClassType getClassType() const override { return EIntegrator; }
};
struct PathMats : Integrator { explicit PathMats(const PropertyList &) : Integrator(NORI_INTEGRATOR_PATH_MATS) {} };
NORI_REGISTER_CLASS(PathMats, "path_mats")
struct PathMis : Integrator { explicit PathMis(const PropertyList &) : Integrator(NORI_INTEGRATOR_PATH_MIS) {} };
NORI_REGISTER_CLASS(PathMis, "path_mis")
struct Volumetric : Integrator { explicit Volumetric(const PropertyList &) : Integrator(NORI_INTEGRATOR_VOLUMETRIC) {} };
NORI_REGISTER_CLASS(Volumetric, "volumetric")
struct Normals : Integrator { explicit Normals(const PropertyList &) : Integrator(NORI_INTEGRATOR_NORMALS) {} };
NORI_REGISTER_CLASS(Normals, "normals")
struct AverageVisibility : Integrator {  // averagevisibility.cpp:11-14
    float length;
    explicit AverageVisibility(const PropertyList &p) : Integrator(NORI_INTEGRATOR_AV), length(p.getFloat("length")) {}
};
NORI_REGISTER_CLASS(AverageVisibility, "av")
struct Direct : Integrator { explicit Direct(const PropertyList &) : Integrator(NORI_INTEGRATOR_DIRECT) {} };
NORI_REGISTER_CLASS(Direct, "direct")
struct DirectEms : Integrator { explicit DirectEms(const PropertyList &) : Integrator(NORI_INTEGRATOR_DIRECT_EMS) {} };
NORI_REGISTER_CLASS(DirectEms, "direct_ems")
struct DirectMats : Integrator { explicit DirectMats(const PropertyList &) : Integrator(NORI_INTEGRATOR_DIRECT_MATS) {} };
NORI_REGISTER_CLASS(DirectMats, "direct_mats")
struct DirectMis : Integrator { explicit DirectMis(const PropertyList &) : Integrator(NORI_INTEGRATOR_DIRECT_MIS) {} };
NORI_REGISTER_CLASS(DirectMis, "direct_mis")
struct PhotonMapper : Integrator {  // photonmapper.cpp:34-39
    int count;
    float radius;
    explicit PhotonMapper(const PropertyList &p)
        : Integrator(NORI_INTEGRATOR_PHOTONMAPPER), count(p.getInteger("photonCount", 1000000)),
          radius(p.getFloat("photonRadius", 0.0f)) {}
};
NORI_REGISTER_CLASS(PhotonMapper, "photonmapper")
struct Phase : NoriObject {
    explicit Phase(const PropertyList &) {}
    EClassType getClassType() const override { return EPhaseFunction; }
};
NORI_REGISTER_CLASS(Phase, "isotropic")
struct Medium : NoriObject {  // medium.cpp:5-19
    nori_medium_desc d{};
    NoriObject *phase = nullptr;
    explicit Medium(const PropertyList &p) {
        d.present = 1;
        Vec3f a = p.getColor("sigma_a"), s = p.getColor("sigma_s");
        Vec3f sz = p.getVector3("box_size"), o = p.getVector3("box_origin");
        sz = Vec3f{std::fabs(sz.x), std::fabs(sz.y), std::fabs(sz.z)};
        d.sigma_a[0] = a.x; d.sigma_a[1] = a.y; d.sigma_a[2] = a.z;
        d.sigma_s[0] = s.x; d.sigma_s[1] = s.y; d.sigma_s[2] = s.z;
        d.box_min[0] = o.x - sz.x; d.box_min[1] = o.y - sz.y; d.box_min[2] = o.z - sz.z;
        d.box_max[0] = o.x + sz.x; d.box_max[1] = o.y + sz.y; d.box_max[2] = o.z + sz.z;
    }
    ~Medium() override { delete phase; }
    EClassType getClassType() const override { return EMedium; }
    void addChild(NoriObject *o) override {  // medium.cpp:104-115
        if (o->getClassType() != EPhaseFunction) throw NoriException(NORI_ERR_PARSE, "Can only register a phase function");
        if (phase) throw NoriException(NORI_ERR_PARSE, "Phase function already registered");
        phase = o;
    }
};
NORI_REGISTER_CLASS(Medium, "medium")

// ---- scene (scene.cpp)
struct SceneObj : NoriObject {
    std::vector<Shape *> shapes;
    std::vector<Emitter *> emitters;  // addChild order (scene.cpp:63-77)
    std::vector<Emitter *> free_emitters;  // owned here (shape emitters are owned by their shape)
    Independent *sampler = nullptr;
    Perspective *camera = nullptr;
    Integrator *integrator = nullptr;
    Medium *medium = nullptr;
    explicit SceneObj(const PropertyList &) {}
    ~SceneObj() override {
        for (auto *s : shapes) { if (s->emitter) { delete s->emitter; s->emitter = nullptr; } delete s; }
        for (auto *e : free_emitters) delete e;
        delete sampler; delete camera; delete integrator; delete medium;
    }
    EClassType getClassType() const override { return EScene; }
    void addChild(NoriObject *o) override {
        switch (o->getClassType()) {
        case EMesh: {
            auto *m = static_cast<Shape *>(o);
            shapes.push_back(m);
            if (m->emitter) emitters.push_back(m->emitter);
            break;
        }
        case EEmitter:  // free-standing emitters (scene.cpp:73-75)
            emitters.push_back(static_cast<Emitter *>(o));
            free_emitters.push_back(static_cast<Emitter *>(o));
            break;
        case ESampler:
            if (sampler) throw NoriException(NORI_ERR_PARSE, "There can only be one sampler per scene!");
            sampler = static_cast<Independent *>(o);
            break;
        case ECamera:
            if (camera) throw NoriException(NORI_ERR_PARSE, "There can only be one camera per scene!");
            camera = static_cast<Perspective *>(o);
            break;
        case EIntegrator:
            if (integrator) throw NoriException(NORI_ERR_PARSE, "There can only be one integrator per scene!");
            integrator = static_cast<Integrator *>(o);
            break;
        case EMedium:
            delete medium;
            medium = static_cast<Medium *>(o);
            break;
        default:
            throw NoriException(NORI_ERR_PARSE, std::string("Scene::addChild(<") + class_name(o->getClassType()) + ">) is not supported!");
        }
    }
    void activate() override {  // scene.cpp:43-61
        if (!integrator) throw NoriException(NORI_ERR_PARSE, "No integrator was specified!");
        if (!camera) throw NoriException(NORI_ERR_PARSE, "No camera was specified!");
        if (!sampler) {
            sampler = static_cast<Independent *>(registry().at("independent")(PropertyList()));
            sampler->activate();
        }
    }
};
NORI_REGISTER_CLASS(SceneObj, "scene")

// ------------------------------------------------------------------ loadFromXML (parser.cpp:28-338)
enum ETag {
    TBoolean = EClassTypeCount, TInteger, TFloat, TString, TPoint, TVector, TColor, TTransform, TTranslate, TMatrix,
    TRotate, TScale, TLookAt, TInvalid
};

static NoriObject *parse_tag(const XmlNode &node, PropertyList &list, int parentTag, Mat4 &transform,
                             const std::string &file) {
    static const std::map<std::string, int> tags = {
        {"scene", EScene}, {"mesh", EMesh}, {"texture", ETexture}, {"bsdf", EBSDF}, {"emitter", EEmitter},
        {"camera", ECamera}, {"medium", EMedium}, {"phase", EPhaseFunction}, {"integrator", EIntegrator},
        {"sampler", ESampler}, {"rfilter", EReconstructionFilter}, {"test", ETest}, {"boolean", TBoolean},
        {"integer", TInteger}, {"float", TFloat}, {"string", TString}, {"point", TPoint}, {"vector", TVector},
        {"color", TColor}, {"transform", TTransform}, {"translate", TTranslate}, {"matrix", TMatrix},
        {"rotate", TRotate}, {"scale", TScale}, {"lookat", TLookAt}};
    auto where = [&](const std::string &m) {
        return "Error while parsing \"" + file + "\": " + m + " (at row " + std::to_string(node.line) + ")";
    };
    auto it = tags.find(node.name);
    if (it == tags.end()) throw NoriException(NORI_ERR_PARSE, where("unexpected tag \"" + node.name + "\""));
    int tag = it->second;
    bool hasParent = parentTag != TInvalid;
    bool parentIsObject = hasParent && parentTag < EClassTypeCount;
    bool currentIsObject = tag < EClassTypeCount;
    bool parentIsTransform = parentTag == TTransform;
    bool currentIsTransformOp = tag == TTranslate || tag == TRotate || tag == TScale || tag == TLookAt || tag == TMatrix;
    if (!hasParent && !currentIsObject)
        throw NoriException(NORI_ERR_PARSE, where("root element \"" + node.name + "\" must be a Nori object"));
    if (parentIsTransform != currentIsTransformOp)
        throw NoriException(NORI_ERR_PARSE, where("transform nodes can only contain transform operations"));
    if (hasParent && !parentIsObject && !(parentIsTransform && currentIsTransformOp))
        throw NoriException(NORI_ERR_PARSE, where("node \"" + node.name + "\" requires a Nori object as parent"));
    if (tag == TTransform) transform = mat_identity();

    PropertyList props;
    std::vector<std::unique_ptr<NoriObject>> children;
    for (auto &ch : node.children) {
        NoriObject *c = parse_tag(ch, props, tag, transform, file);
        if (c) children.emplace_back(c);
    }
    auto attr = [&](const char *k) -> std::string {
        const std::string *v = node.attr(k);
        if (!v) throw NoriException(NORI_ERR_PARSE, where(std::string("missing attribute \"") + k + "\" in \"" + node.name + "\""));
        return *v;
    };
    try {
        if (currentIsObject) {
            std::string type = tag == EScene ? "scene" : (node.attr("type") ? *node.attr("type") : "");
            if (tag == ETest) throw NoriException(NORI_ERR_UNSUPPORTED, "test harness roots are driven by tests/, not the renderer");
            auto ct = registry().find(type);
            if (ct == registry().end()) {
                for (const char *u : kUnsupported)
                    if (type == u) throw NoriException(NORI_ERR_UNSUPPORTED, "plugin \"" + type + "\" is outside this path's scope");
                throw NoriException(NORI_ERR_PARSE, "A constructor for class \"" + type + "\" could not be found!");
            }
            std::unique_ptr<NoriObject> result(ct->second(props));
            if (result->getClassType() != tag)
                throw NoriException(NORI_ERR_PARSE, std::string("Unexpectedly constructed an object of type <") +
                                                        class_name(result->getClassType()) + "> (expected type <" +
                                                        class_name(tag) + ">)");
            if (const std::string *nm = node.attr("name")) result->idName = *nm;
            for (auto &c : children) {
                NoriObject *raw = c.release();
                result->addChild(raw);
                raw->setParent(result.get());
            }
            result->activate();
            return result.release();
        }
        Property p;
        switch (tag) {
        case TString: p.type = Property::String; p.s = attr("value"); list.set(attr("name"), p); break;
        case TFloat: p.type = Property::Float; p.f = to_float(attr("value")); list.set(attr("name"), p); break;
        case TInteger: p.type = Property::Int; p.i = to_int(attr("value")); list.set(attr("name"), p); break;
        case TBoolean: p.type = Property::Bool; p.b = to_bool(attr("value")); list.set(attr("name"), p); break;
        case TPoint:
        case TVector: {
            auto t = tokenize(attr("value"));
            if (t.size() == 3) { p.type = tag == TPoint ? Property::Point3 : Property::Vector3; p.v = to_vec3(attr("value")); }
            else if (t.size() == 2) { p.type = tag == TPoint ? Property::Point2 : Property::Vector2; p.v2[0] = to_float(t[0]); p.v2[1] = to_float(t[1]); }
            else throw NoriException(NORI_ERR_PARSE, "Point/Vector " + attr("name") + " is not of size 2 or 3");
            list.set(attr("name"), p);
            break;
        }
        case TColor: p.type = Property::Color; p.v = to_vec3(attr("value")); list.set(attr("name"), p); break;
        case TTransform: p.type = Property::Transform; p.t = transform; list.set(attr("name"), p); break;
        case TTranslate: {
            Vec3f v = to_vec3(attr("value"));
            Mat4 t = mat_identity(); t.m[3] = v.x; t.m[7] = v.y; t.m[11] = v.z;
            transform = mat_mul(t, transform);
            break;
        }
        case TMatrix: {
            auto t = tokenize(attr("value"));
            if (t.size() != 16) throw NoriException(NORI_ERR_PARSE, "Expected 16 values");
            Mat4 m;
            for (int i = 0; i < 16; ++i) m.m[i] = to_float(t[i]);
            transform = mat_mul(m, transform);
            break;
        }
        case TScale: {
            Vec3f v = to_vec3(attr("value"));
            Mat4 s = mat_identity(); s.m[0] = v.x; s.m[5] = v.y; s.m[10] = v.z;
            transform = mat_mul(s, transform);
            break;
        }
        case TRotate: {  // Eigen::AngleAxis<float>::toRotationMatrix
            float angle = to_float(attr("angle")) * (3.14159265358979323846f / 180.0f);
            Vec3f a = to_vec3(attr("axis"));
            float sn = std::sin(angle), c = std::cos(angle);
            Vec3f sa{sn * a.x, sn * a.y, sn * a.z}, ca{(1.0f - c) * a.x, (1.0f - c) * a.y, (1.0f - c) * a.z};
            Mat4 r = mat_identity();
            float tmp = ca.x * a.y; r.m[1] = tmp - sa.z; r.m[4] = tmp + sa.z;
            tmp = ca.x * a.z; r.m[2] = tmp + sa.y; r.m[8] = tmp - sa.y;
            tmp = ca.y * a.z; r.m[6] = tmp - sa.x; r.m[9] = tmp + sa.x;
            r.m[0] = ca.x * a.x + c; r.m[5] = ca.y * a.y + c; r.m[10] = ca.z * a.z + c;
            transform = mat_mul(r, transform);
            break;
        }
        case TLookAt: {  // parser.cpp:307-322
            Vec3f o = to_vec3(attr("origin")), tg = to_vec3(attr("target")), up = to_vec3(attr("up"));
            Vec3f dir = normalized(Vec3f{tg.x - o.x, tg.y - o.y, tg.z - o.z});
            Vec3f left = normalized(vcross(normalized(up), dir));
            Vec3f nup = normalized(vcross(dir, left));
            Mat4 t = mat_identity();
            t.m[0] = left.x; t.m[4] = left.y; t.m[8] = left.z;
            t.m[1] = nup.x; t.m[5] = nup.y; t.m[9] = nup.z;
            t.m[2] = dir.x; t.m[6] = dir.y; t.m[10] = dir.z;
            t.m[3] = o.x; t.m[7] = o.y; t.m[11] = o.z;
            transform = mat_mul(t, transform);
            break;
        }
        default:
            throw NoriException(NORI_ERR_PARSE, "Unhandled element \"" + node.name + "\"");
        }
    } catch (const NoriException &e) {
        if (std::string(e.what()).rfind("Error while parsing", 0) == 0) throw;
        throw NoriException(e.code, where(e.what()));
    }
    return nullptr;
}

static thread_local std::string g_base_dir;
std::string resolve_path(const std::string &p) {  // filesystem::resolver: scene directory first
    if (!p.empty() && p[0] == '/') return p;
    if (!g_base_dir.empty()) {
        std::string c = g_base_dir + "/" + p;
        std::ifstream t(c);
        if (t.good()) return c;
    }
    return p;
}

// ------------------------------------------------------------------ flattening
HostScene *load_scene_xml(const std::string &path, int width, int height, int spp) {
    std::ifstream is(path, std::ios::binary);
    if (!is) throw NoriException(NORI_ERR_IO, "Unable to open scene file \"" + path + "\"");
    std::stringstream ss;
    ss << is.rdbuf();
    std::string text = ss.str();
    size_t slash = path.find_last_of('/');
    g_base_dir = slash == std::string::npos ? "." : path.substr(0, slash);
    XmlNode root = XmlParser(text, path).parse();
    PropertyList dummy;
    Mat4 xf = mat_identity();
    std::unique_ptr<NoriObject> obj(parse_tag(root, dummy, TInvalid, xf, path));
    if (!obj || obj->getClassType() != EScene)
        throw NoriException(NORI_ERR_UNSUPPORTED, "the XML root is not a <scene>");
    auto *sc = static_cast<SceneObj *>(obj.get());

    auto hs = std::make_unique<HostScene>();
    hs->source = path;
    std::vector<const ImageTex *> image_src;  // one images[] entry per texture object
    auto add_image = [&](const ImageTex *t) -> int32_t {
        for (size_t i = 0; i < image_src.size(); ++i)
            if (image_src[i] == t) return (int32_t)i;
        image_src.push_back(t);
        hs->image_rgb.push_back(t->rgb);
        hs->images.push_back(nori_image_desc{t->width, t->height, t->wrap, nullptr});
        return (int32_t)(image_src.size() - 1);
    };
    for (size_t si = 0; si < sc->shapes.size(); ++si) {
        Shape *sh = sc->shapes[si];
        nori_shape_desc d{};
        d.emitter = -1;
        d.normal_map = sh->normal_map ? add_image(sh->normal_map) : -1;
        d.bsdf = (int32_t)hs->bsdfs.size();
        const Bsdf *bo = static_cast<Bsdf *>(sh->bsdf);
        hs->bsdfs.push_back(bo->d);
        hs->bsdfs.back().albedo_image = bo->image ? add_image(bo->image) : -1;
        if (auto *m = dynamic_cast<WavefrontOBJ *>(sh)) {
            d.type = NORI_SHAPE_MESH;
            d.vtx_offset = (uint32_t)(hs->positions.size() / 3);
            d.vtx_count = (uint32_t)(m->V.size() / 3);
            d.tri_offset = (uint32_t)(hs->indices.size() / 3);
            d.tri_count = (uint32_t)(m->F.size() / 3);
            d.has_normals = !m->N.empty();
            d.has_uvs = !m->UV.empty();
            hs->positions.insert(hs->positions.end(), m->V.begin(), m->V.end());
            if (d.has_normals) hs->normals.insert(hs->normals.end(), m->N.begin(), m->N.end());
            else hs->normals.insert(hs->normals.end(), m->V.size(), 0.0f);
            if (d.has_uvs) hs->uvs.insert(hs->uvs.end(), m->UV.begin(), m->UV.end());
            else hs->uvs.insert(hs->uvs.end(), 2 * (m->V.size() / 3), 0.0f);
            for (uint32_t f : m->F) hs->indices.push_back(f + d.vtx_offset);
            // bbox over every OBJ vertex (obj.cpp:62), used as the BVH root box
            for (size_t v = 0; v < m->V.size(); v += 3) hs->expand_root(m->V[v], m->V[v + 1], m->V[v + 2]);
        } else {
            auto *s = static_cast<Sphere *>(sh);
            d.type = NORI_SHAPE_SPHERE;
            d.tri_count = 1;
            d.center[0] = s->center.x; d.center[1] = s->center.y; d.center[2] = s->center.z;
            d.radius = s->radius;
            hs->expand_root(s->center.x - s->radius, s->center.y - s->radius, s->center.z - s->radius);
            hs->expand_root(s->center.x + s->radius, s->center.y + s->radius, s->center.z + s->radius);
        }
        hs->shapes.push_back(d);
    }
    for (Emitter *e : sc->emitters) {
        nori_emitter_desc ed = e->d;
        if (ed.type == NORI_EMITTER_ENVMAP) {
            hs->env_images.push_back(e->rgb);
            ed.env_rgb = hs->env_images.back().data();
        }
        for (size_t si = 0; si < sc->shapes.size(); ++si)
            if (sc->shapes[si]->emitter == e) {
                ed.shape = (int32_t)si;
                hs->shapes[si].emitter = (int32_t)hs->emitters.size();
            }
        hs->emitters.push_back(ed);
    }
    const int integ = sc->integrator->kind;
    // normals and av never query emitters; every other integrator samples one
    // (Scene::getRandomEmitter on an empty list is undefined, scene.h:68-74)
    if (hs->emitters.empty() && integ != NORI_INTEGRATOR_NORMALS && integ != NORI_INTEGRATOR_AV)
        throw NoriException(NORI_ERR_INVALID, "the scene has no emitter");
    if (integ == NORI_INTEGRATOR_AV) hs->desc.av_length = static_cast<AverageVisibility *>(sc->integrator)->length;
    if (integ == NORI_INTEGRATOR_PHOTONMAPPER) {
        auto *pm = static_cast<PhotonMapper *>(sc->integrator);
        if (pm->count <= 0) throw NoriException(NORI_ERR_INVALID, "photonmapper: photonCount must be positive");
        for (const nori_emitter_desc &e : hs->emitters)  // Emitter::samplePhoton (emitter.h:106-108)
            if (e.type != NORI_EMITTER_AREA)
                throw NoriException(NORI_ERR_UNSUPPORTED, "Emitter::samplePhoton(): not implemented!");
        float r = pm->radius;
        if (r == 0) {  // photonmapper.cpp:55-56: scene bounding box diagonal / 500
            const float e0 = hs->root_max[0] - hs->root_min[0], e1 = hs->root_max[1] - hs->root_min[1],
                        e2 = hs->root_max[2] - hs->root_min[2];
            r = std::sqrt((e0 * e0 + e1 * e1) + e2 * e2) / 500.0f;
        }
        hs->desc.photon_count = (uint32_t)pm->count;
        hs->desc.photon_radius = r;
    }
    nori_camera_desc cam = sc->camera->d;
    if (width > 0) cam.width = width;
    if (height > 0) cam.height = height;
    compute_sample_to_camera(cam);
    cam.filter_type = sc->camera->filter->type;
    cam.filter_radius = sc->camera->filter->radius;
    cam.filter_p0 = sc->camera->filter->p0;
    cam.filter_p1 = sc->camera->filter->p1;
    hs->desc.camera = cam;
    hs->desc.integrator = sc->integrator->kind;
    if (sc->medium) hs->desc.medium = sc->medium->d;
    if (hs->desc.integrator == NORI_INTEGRATOR_VOLUMETRIC && !sc->medium)
        throw NoriException(NORI_ERR_INVALID, "the volumetric integrator needs a <medium> (scene.h:141 leaves it unset)");
    hs->desc.sample_count = (uint32_t)(spp > 0 ? spp : sc->sampler->sampleCount);
    hs->finalize();
    return hs.release();
}

void HostScene::finalize() {
    desc.abi_version = NORI_GPU_ABI_VERSION;
    desc.num_vertices = (uint32_t)(positions.size() / 3);
    desc.positions = positions.data();
    desc.normals = normals.data();
    desc.uvs = uvs.data();
    desc.num_triangles = (uint32_t)(indices.size() / 3);
    desc.indices = indices.data();
    desc.num_shapes = (uint32_t)shapes.size();
    desc.shapes = shapes.data();
    desc.num_bsdfs = (uint32_t)bsdfs.size();
    desc.bsdfs = bsdfs.data();
    desc.num_emitters = (uint32_t)emitters.size();
    desc.emitters = emitters.data();
    for (size_t i = 0; i < images.size(); ++i) images[i].rgb = image_rgb[i].data();
    desc.num_images = (uint32_t)images.size();
    desc.images = images.data();
}

}  // namespace nori
