// collada.cpp -- the reference's Collada path, ColladaLoader::load
// (ColladaLoader.cpp:13-593) + Mesh::init(ColladaLoader&) (Mesh.cpp:10-78),
// in linear time, plus the writer of that subset (the synthetic-scene DAE
// generator of SURVEY.md 8d).
//
// The reference parses with pugixml (not vendored, README:4) and walks the DOM
// with child()/next_sibling() lookups; this file has its own small DOM parser
// with the pugixml behaviours the loader depends on: element text() is the
// first non-whitespace PCDATA / CDATA child, unmodified (no trimming); entity
// and character references are decoded; a missing node or attribute reads as
// "" (as_int -> 0).  Numbers are read as the reference reads them: float
// arrays by successive std::stof (strtof, correctly rounded), <p> by
// sscanf("%d" x 9), count by sscanf("%d").
//
// Reference quirks kept on purpose (they decide the output):
//  * effects are keyed by their `name` attribute; an effect without
//    cook-torrance / phong still takes its index but is not appended
//    (ColladaLoader.cpp:119-131 / :183-186), so later indices shift;
//  * a <polygons material> or <instance_geometry url> that names nothing maps
//    to index 0 (unordered_map::operator[]);
//  * <p> holds exactly 9 ints in VERTEX/NORMAL/TEXCOORD order whatever the
//    input offsets (:421-427); missing <p> elements leave zero indices;
//  * only the first 3 <input>s of <polygons> are searched (:408-419), and all
//    three semantics must be present (`.substr(1)` of "" throws, :233-235);
//  * node transform: <matrix> (transposed) if present, else the rotates keyed
//    by sid in the order jointOrientX/Y/Z, rotateX, rotateZ, rotateY applied as
//    rotateX, rotateY, rotateZ, rotateX, rotateY, rotateZ (i % 3, :488-520) --
//    so sid "rotateZ" rotates about Y -- then translate; the angle text skips
//    its first 6 characters (the axis, :503);
//  * geometry g takes the transform of the LAST of the first G scene nodes
//    that instances it, scene node 0 if none (:583-592);
//  * normals are transformed with w = 0 and stored with w = 1, not normalized
//    (Mesh.cpp:66-73); the scene box starts at the first vertex (:50-57).
// Deviations: sin/cos of the rotation angle are (float)sin((double)a) (MSVC's
// sinf is not available here; results agree except possibly in the last bit
// for some angles); a node without <translate> translates by 0 (the reference
// reads uninitialised floats); malformed input is reported instead of
// crashing.
#include <algorithm>
#include <cctype>
#include <cerrno>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <string>
#include <unordered_map>
#include <vector>

#include "scene.hpp"

namespace rtamd {
namespace {

// ---------------------------------------------------------------- XML DOM
struct XNode {
    std::string name;
    std::vector<std::pair<std::string, std::string>> attrs;
    int32_t first_child = -1, next_sibling = -1, parent = -1;
    // first PCDATA/CDATA child's text: [text_off, text_off + text_len) of Doc::buf,
    // or the decoded copy in `text_own` when it held references
    int64_t text_off = -1, text_len = 0;
    std::string text_own;
    bool text_decoded = false;
};

struct Doc {
    std::string buf;
    std::vector<XNode> nodes;  // node 0 = document
    std::string err;

    const XNode* child(const XNode* n, const char* name) const {
        if (!n) return nullptr;
        for (int32_t c = n->first_child; c >= 0; c = nodes[c].next_sibling)
            if (nodes[c].name == name) return &nodes[c];
        return nullptr;
    }
    const XNode* next(const XNode* n, const char* name) const {
        if (!n) return nullptr;
        for (int32_t c = n->next_sibling; c >= 0; c = nodes[c].next_sibling)
            if (nodes[c].name == name) return &nodes[c];
        return nullptr;
    }
    const XNode* parent(const XNode* n) const { return (n && n->parent >= 0) ? &nodes[n->parent] : nullptr; }
    static const char* attr(const XNode* n, const char* name) {
        if (!n) return "";
        for (const auto& a : n->attrs)
            if (a.first == name) return a.second.c_str();
        return "";
    }
    // text().as_string(): a C string (points into buf: terminated by the '<' that
    // follows; callers parse numbers, which stop there)
    std::string text(const XNode* n) const {
        if (!n || n->text_off < 0) return std::string();
        if (n->text_decoded) return n->text_own;
        return buf.substr((size_t)n->text_off, (size_t)n->text_len);
    }
    const char* text_ptr(const XNode* n, size_t& len) const {
        if (!n || n->text_off < 0) { len = 0; return ""; }
        if (n->text_decoded) { len = n->text_own.size(); return n->text_own.c_str(); }
        len = (size_t)n->text_len;
        return buf.data() + n->text_off;
    }
};

bool is_ws(char c) { return c == ' ' || c == '\t' || c == '\n' || c == '\r'; }

bool decode_refs(const char* s, size_t n, std::string& out) {
    out.clear();
    out.reserve(n);
    for (size_t i = 0; i < n; ++i) {
        if (s[i] != '&') { out.push_back(s[i]); continue; }
        const char* e = (const char*)std::memchr(s + i, ';', n - i);
        if (!e) { out.push_back('&'); continue; }
        const std::string ent(s + i + 1, e - (s + i + 1));
        unsigned long cp = 0;
        bool ok = true;
        if (ent == "lt") cp = '<';
        else if (ent == "gt") cp = '>';
        else if (ent == "amp") cp = '&';
        else if (ent == "quot") cp = '"';
        else if (ent == "apos") cp = '\'';
        else if (ent.size() > 1 && ent[0] == '#') cp = (ent[1] == 'x') ? std::strtoul(ent.c_str() + 2, nullptr, 16)
                                                                        : std::strtoul(ent.c_str() + 1, nullptr, 10);
        else ok = false;
        if (!ok) { out.push_back('&'); continue; }
        if (cp < 0x80) out.push_back((char)cp);
        else if (cp < 0x800) { out.push_back((char)(0xC0 | (cp >> 6))); out.push_back((char)(0x80 | (cp & 0x3F))); }
        else if (cp < 0x10000) {
            out.push_back((char)(0xE0 | (cp >> 12))); out.push_back((char)(0x80 | ((cp >> 6) & 0x3F)));
            out.push_back((char)(0x80 | (cp & 0x3F)));
        } else {
            out.push_back((char)(0xF0 | (cp >> 18))); out.push_back((char)(0x80 | ((cp >> 12) & 0x3F)));
            out.push_back((char)(0x80 | ((cp >> 6) & 0x3F))); out.push_back((char)(0x80 | (cp & 0x3F)));
        }
        i = (size_t)(e - s);
    }
    return true;
}

bool parse_xml(Doc& d) {
    const std::string& b = d.buf;
    const size_t n = b.size();
    d.nodes.clear();
    d.nodes.emplace_back();  // document
    std::vector<int32_t> open{0};
    std::vector<int32_t> last_child{-1};
    size_t i = 0;
    auto add_node = [&](XNode&& x) -> int32_t {
        const int32_t id = (int32_t)d.nodes.size();
        x.parent = open.back();
        d.nodes.push_back(std::move(x));
        if (last_child.back() < 0) d.nodes[open.back()].first_child = id;
        else d.nodes[last_child.back()].next_sibling = id;
        last_child.back() = id;
        return id;
    };
    auto set_text = [&](size_t off, size_t len, bool may_have_refs) {
        XNode& p = d.nodes[open.back()];
        if (p.text_off >= 0) return;  // text() = first PCDATA child
        if (may_have_refs && std::memchr(b.data() + off, '&', len)) {
            decode_refs(b.data() + off, len, p.text_own);
            p.text_decoded = true;
        }
        p.text_off = (int64_t)off;
        p.text_len = (int64_t)len;
    };
    while (i < n) {
        if (b[i] != '<') {
            const size_t s = i;
            while (i < n && b[i] != '<') ++i;
            bool ws = true;
            for (size_t k = s; k < i && ws; ++k) ws = is_ws(b[k]);
            if (!ws && open.size() > 1) set_text(s, i - s, true);
            continue;
        }
        if (b.compare(i, 4, "<!--") == 0) {
            const size_t e = b.find("-->", i + 4);
            if (e == std::string::npos) { d.err = "unterminated comment"; return false; }
            i = e + 3;
            continue;
        }
        if (b.compare(i, 9, "<![CDATA[") == 0) {
            const size_t e = b.find("]]>", i + 9);
            if (e == std::string::npos) { d.err = "unterminated CDATA"; return false; }
            if (open.size() > 1) set_text(i + 9, e - (i + 9), false);
            i = e + 3;
            continue;
        }
        if (b.compare(i, 2, "<?") == 0) {
            const size_t e = b.find("?>", i + 2);
            if (e == std::string::npos) { d.err = "unterminated declaration"; return false; }
            i = e + 2;
            continue;
        }
        if (b.compare(i, 2, "<!") == 0) {  // DOCTYPE and friends (no internal subset support)
            const size_t e = b.find('>', i + 2);
            if (e == std::string::npos) { d.err = "unterminated <!"; return false; }
            i = e + 1;
            continue;
        }
        if (b.compare(i, 2, "</") == 0) {
            const size_t e = b.find('>', i + 2);
            if (e == std::string::npos || open.size() <= 1) { d.err = "bad end tag"; return false; }
            open.pop_back();
            last_child.pop_back();
            i = e + 1;
            continue;
        }
        // start tag
        ++i;
        XNode x;
        const size_t ns = i;
        while (i < n && !is_ws(b[i]) && b[i] != '>' && b[i] != '/') ++i;
        x.name.assign(b, ns, i - ns);
        bool self_close = false;
        for (;;) {
            while (i < n && is_ws(b[i])) ++i;
            if (i >= n) { d.err = "unterminated tag"; return false; }
            if (b[i] == '>') { ++i; break; }
            if (b[i] == '/') { self_close = true; i = b.find('>', i); if (i == std::string::npos) return false; ++i; break; }
            const size_t as = i;
            while (i < n && !is_ws(b[i]) && b[i] != '=' && b[i] != '>') ++i;
            std::string an(b, as, i - as);
            while (i < n && is_ws(b[i])) ++i;
            if (i >= n || b[i] != '=') { d.err = "attribute without value"; return false; }
            ++i;
            while (i < n && is_ws(b[i])) ++i;
            if (i >= n || (b[i] != '"' && b[i] != '\'')) { d.err = "unquoted attribute"; return false; }
            const char q = b[i++];
            const size_t vs = i;
            while (i < n && b[i] != q) ++i;
            if (i >= n) { d.err = "unterminated attribute"; return false; }
            std::string v;
            decode_refs(b.data() + vs, i - vs, v);
            for (char& c : v) if (c == '\t' || c == '\n' || c == '\r') c = ' ';  // parse_wconv_attribute
            ++i;
            x.attrs.emplace_back(std::move(an), std::move(v));
        }
        const int32_t id = add_node(std::move(x));
        if (!self_close) {
            open.push_back(id);
            last_child.push_back(-1);
        }
    }
    if (open.size() != 1) { d.err = "unclosed elements"; return false; }
    return true;
}

// ---------------------------------------------------------------- numbers
// stof_array (ColladaLoader.h:20-31): successive std::stof over the text.
bool stof_array(const char* s, size_t len, int n, float* out) {
    if (len < 1 || n < 1 || !out) return true;  // "returns 0": nothing written
    const char* p = s;
    for (int i = 0; i < n; ++i) {
        char* e = nullptr;
        errno = 0;
        const float f = std::strtof(p, &e);
        if (e == p) return false;                // std::invalid_argument
        if (errno == ERANGE) return false;       // std::out_of_range
        out[i] = f;
        p = e;
    }
    return true;
}

int scan_ints(const char* s, int n, int32_t* out) {  // sscanf("%d ...")
    const char* p = s;
    int k = 0;
    for (; k < n; ++k) {
        while (*p && std::isspace((unsigned char)*p)) ++p;
        char* e = nullptr;
        const long v = std::strtol(p, &e, 10);
        if (e == p) break;
        out[k] = (int32_t)v;
        p = e;
    }
    return k;
}

// ---------------------------------------------------------------- Matrix4x4 (Matrix4x4.cpp)
struct Mat4 {
    float m[16];
    Mat4() { set_identity(); }
    void set_identity() { for (int i = 0; i < 16; ++i) m[i] = (i % 5 == 0) ? 1.0f : 0.0f; }
    void mul(const Mat4& b) {  // this = this * b, row-major, k-sum from 0
        Mat4 r;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) {
                float s = 0.0f;
                for (int k = 0; k < 4; ++k) s += m[i * 4 + k] * b.m[k * 4 + j];
                r.m[i * 4 + j] = s;
            }
        *this = r;
    }
    void transpose() {
        Mat4 r;
        for (int i = 0; i < 4; ++i)
            for (int j = 0; j < 4; ++j) r.m[j * 4 + i] = m[i * 4 + j];
        *this = r;
    }
    static Mat4 rows(std::initializer_list<float> v) {
        Mat4 r;
        int i = 0;
        for (float x : v) r.m[i++] = x;
        return r;
    }
    void rotate(int axis, float a) {  // rotateX / rotateY / rotateZ
        const float s = (float)std::sin((double)a), c = (float)std::cos((double)a);
        if (axis == 0) mul(rows({1, 0, 0, 0, 0, c, s, 0, 0, -s, c, 0, 0, 0, 0, 1}));
        else if (axis == 1) mul(rows({c, 0, -s, 0, 0, 1, 0, 0, s, 0, c, 0, 0, 0, 0, 1}));
        else mul(rows({c, s, 0, 0, -s, c, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1}));
    }
    void translate(float x, float y, float z) { mul(rows({1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, x, y, z, 1})); }
    void apply(const float v[4], float out[4]) const {  // multiply(float4, Matrix4x4) (Matrix4x4.h:38-52)
        for (int i = 0; i < 4; ++i) {
            float s = 0.0f;
            for (int j = 0; j < 4; ++j) s += v[j] * m[j * 4 + i];
            out[i] = s;
        }
    }
};

// ---------------------------------------------------------------- ColladaLoader
const char* kAttr[10] = {"emission", "ambient", "diffuse", "specular", "shininess",
                         "reflective", "reflectivity", "transparent", "transparency", "glossiness"};
const int kAttrN[10] = {4, 4, 4, 4, 1, 4, 1, 4, 1, 1};
const char* kAttrSub[10] = {"color", "color", "color", "color", "float", "color", "float", "color", "float", "float"};

struct Tri9 { int32_t v[3], nrm[3], uv[3]; int32_t effect; };
struct Geometry {
    std::vector<float> pos, nrm, uv;  // float3 / float3 / float2 arrays
    std::vector<Tri9> polys;
};
struct SceneNode { int32_t geometry; Mat4 matrix; };

struct Loader {
    const Doc& d;
    std::string err;
    std::unordered_map<std::string, int> effect_index, geometry_index;
    std::vector<rt_material> effects;
    std::vector<Geometry> geometries;
    std::vector<SceneNode> scene;
    explicit Loader(const Doc& doc) : d(doc) {}

    bool floats(const XNode* n, int count, float* out) {
        size_t len;
        const char* s = d.text_ptr(n, len);
        if (!stof_array(s, len, count, out)) { err = "bad float text in <" + (n ? n->name : std::string("?")) + ">"; return false; }
        return true;
    }

    bool load_effect(const XNode* e, int count) {  // :103-160
        effect_index[Doc::attr(e, "name")] = count;
        const XNode* tech = d.child(d.child(e, "profile_COMMON"), "technique");
        const XNode* cur = d.child(tech, "cook-torrance");
        int technique = 2;  // Effect::COOK_TORRANCE
        if (!cur) { cur = d.child(tech, "phong"); technique = 1; }
        if (!cur) return true;  // not appended (index already taken)
        float c[10][4] = {};
        for (int i = 0; i < 10; ++i)
            if (!floats(d.child(d.child(cur, kAttr[i]), kAttrSub[i]), kAttrN[i], c[i])) return false;
        rt_material m;
        std::memset(&m, 0, sizeof(m));
        m.technique = rt_int4{technique, 0, 0, 0};
        m.emission = rt_float4{c[0][0], c[0][1], c[0][2], c[0][3]};
        m.ambient = rt_float4{c[1][0], c[1][1], c[1][2], c[1][3]};
        m.diffuse = rt_float4{c[2][0], c[2][1], c[2][2], c[2][3]};
        m.specular = rt_float4{c[3][0], c[3][1], c[3][2], c[3][3]};
        m.shininess = rt_float4{c[4][0], 0, 0, 0};
        m.reflective = rt_float4{c[5][0], c[5][1], c[5][2], c[5][3]};
        m.reflectivity = rt_float4{c[6][0], 0, 0, 0};
        m.transparent = rt_float4{c[7][0], c[7][1], c[7][2], c[7][3]};
        m.transparency = rt_float4{c[8][0], 0, 0, 0};
        m.glossiness = rt_float4{c[9][0], 0, 0, 0};
        effects.push_back(m);
        return true;
    }

    std::string input_source(const char* semantic, const XNode* polys) {  // :408-419
        const XNode* in = d.child(polys, "input");
        for (int i = 0; i < 3; ++i) {
            if (in && std::strcmp(Doc::attr(in, "semantic"), semantic) == 0) return Doc::attr(in, "source");
            in = d.next(in, "input");
        }
        return std::string();
    }
    const XNode* float_array(const std::string& id, const XNode* mesh) {  // :383-404
        for (const XNode* s = d.child(mesh, "source"); s; s = d.next(s, "source"))
            if (id == Doc::attr(s, "id")) return d.child(s, "float_array");
        return nullptr;
    }
    std::string vertices_source(const std::string& id, const XNode* mesh) {  // :359-381
        for (const XNode* v = d.child(mesh, "vertices"); v; v = d.next(v, "vertices"))
            if (id == Doc::attr(v, "id")) {
                const std::string s = Doc::attr(d.child(v, "input"), "source");
                return s.empty() ? s : s.substr(1);
            }
        return std::string();
    }
    bool load_array(const XNode* fa, int per, std::vector<float>& out) {  // load_vertices/normals/tex_coords
        const int nf = fa ? std::atoi(Doc::attr(fa, "count")) : 0;
        out.assign((size_t)(std::max(nf, 0) / per) * per, 0.0f);
        if (nf % per) { err = "float_array count not a multiple of " + std::to_string(per); return false; }
        return nf <= 0 || floats(fa, nf, out.data());
    }

    bool load_geometry(const XNode* g, int count) {  // :200-253, load_polygons :255-290
        const XNode* polys = d.child(d.child(g, "mesh"), "polygons");
        geometry_index[Doc::attr(g, "id")] = count;
        Geometry geo;
        int np = 0;
        if (std::sscanf(Doc::attr(polys, "count"), "%d", &np) != 1 || np < 0) {
            err = "<polygons> without a count";
            return false;
        }
        const int effect = effect_index[Doc::attr(polys, "material")];
        geo.polys.assign((size_t)np, Tri9{});
        const XNode* p = d.child(polys, "p");
        for (int i = 0; i < np; ++i) {
            Tri9& t = geo.polys[i];
            t.effect = effect;
            int32_t v9[9] = {0, 0, 0, 0, 0, 0, 0, 0, 0};
            if (p) {
                const std::string s = d.text(p);
                const int k = scan_ints(s.c_str(), 9, v9);
                if (k != 9 && k != 0) { err = "<p> with fewer than 9 indices"; return false; }
            }
            for (int j = 0; j < 3; ++j) { t.v[j] = v9[3 * j]; t.nrm[j] = v9[3 * j + 1]; t.uv[j] = v9[3 * j + 2]; }
            p = d.next(p, "p");
        }
        const XNode* mesh = d.parent(polys);
        const std::string sv = input_source("VERTEX", polys), sn = input_source("NORMAL", polys),
                          st = input_source("TEXCOORD", polys);
        if (sv.empty() || sn.empty() || st.empty()) {
            err = "<polygons> needs VERTEX, NORMAL and TEXCOORD among its first 3 inputs";
            return false;
        }
        const std::string pos_id = vertices_source(sv.substr(1), mesh);
        if (!load_array(float_array(pos_id, mesh), 3, geo.pos)) return false;
        if (!load_array(float_array(sn.substr(1), mesh), 3, geo.nrm)) return false;
        if (!load_array(float_array(st.substr(1), mesh), 2, geo.uv)) return false;
        geometries.push_back(std::move(geo));
        return true;
    }

    bool load_node_matrix(const XNode* node, Mat4& m) {  // :455-545
        m.set_identity();
        if (const XNode* mx = d.child(node, "matrix")) {
            if (!floats(mx, 16, m.m)) return false;
            m.transpose();
            return true;
        }
        std::unordered_map<std::string, const XNode*> rot;
        for (const XNode* r = d.child(node, "rotate"); r; r = d.next(r, "rotate")) rot[Doc::attr(r, "sid")] = r;
        static const char* order[6] = {"jointOrientX", "jointOrientY", "jointOrientZ", "rotateX", "rotateZ", "rotateY"};
        for (int i = 0; i < 6; ++i) {
            auto it = rot.find(order[i]);
            if (it == rot.end()) continue;
            const std::string t = d.text(it->second);
            if (t.size() < 6) { err = "short <rotate>"; return false; }
            float angle = 0.0f;
            const std::string a = t.substr(6);
            if (!stof_array(a.c_str(), a.size(), 1, &angle)) { err = "bad <rotate> angle"; return false; }
            const float rad = (float)((double)angle * 3.14159265358979323846 / 180.0);
            m.rotate(i % 3, rad);
        }
        float tr[3] = {0.0f, 0.0f, 0.0f};
        if (!floats(d.child(node, "translate"), 3, tr)) return false;
        m.translate(tr[0], tr[1], tr[2]);
        return true;
    }

    bool load() {
        const XNode* root = d.child(&d.nodes[0], "COLLADA");
        if (!root) { err = "no <COLLADA> element"; return false; }
        if (const XNode* le = d.child(root, "library_effects")) {
            int c = 0;
            for (const XNode* e = d.child(le, "effect"); e; e = d.next(e, "effect"), ++c)
                if (!load_effect(e, c)) return false;
        }
        if (const XNode* lg = d.child(root, "library_geometries")) {
            int c = 0;
            for (const XNode* g = d.child(lg, "geometry"); g; g = d.next(g, "geometry"), ++c)
                if (!load_geometry(g, c)) return false;
        }
        if (const XNode* vs = d.child(d.child(root, "library_visual_scenes"), "visual_scene")) {
            for (const XNode* nd = d.child(vs, "node"); nd; nd = d.next(nd, "node")) {
                std::string url = Doc::attr(d.child(nd, "instance_geometry"), "url");
                url = url.empty() ? url : url.substr(1);
                SceneNode s;
                s.geometry = geometry_index[url];
                if (!load_node_matrix(nd, s.matrix)) return false;
                scene.push_back(s);
            }
        }
        if (scene.size() < geometries.size()) {  // compute_geometry_to_scene_index reads scene[i], i < G
            err = "fewer visual-scene nodes than geometries";
            return false;
        }
        return true;
    }
};

}  // namespace

int load_dae(const std::string& path, Mesh& m, std::string& err) {
    Doc d;
    {
        std::ifstream f(path, std::ios::binary);
        if (!f) { err = "cannot open " + path; return -1; }
        std::ostringstream ss;
        ss << f.rdbuf();
        d.buf = ss.str();
    }
    // parse_eol: CR LF / CR -> LF (numbers do not care; attribute values do not contain them)
    if (!parse_xml(d)) { err = "XML: " + d.err; return -1; }
    Loader L(d);
    if (!L.load()) { err = L.err; return -1; }

    // Mesh::init(ColladaLoader&) (Mesh.cpp:10-78)
    std::unordered_map<int, int> g2s;  // compute_geometry_to_scene_index (:583-592)
    for (size_t i = 0; i < L.geometries.size(); ++i) g2s[L.scene[i].geometry] = (int)i;
    m = Mesh();
    m.materials = L.effects;
    int32_t vcount = 0, ncount = 0;
    bool first = true;
    for (size_t g = 0; g < L.geometries.size(); ++g) {
        const Geometry& geo = L.geometries[g];
        for (const Tri9& t : geo.polys) {
            for (int j = 0; j < 3; ++j) m.indices.push_back(vcount + t.v[j]);
            for (int j = 0; j < 3; ++j) m.normals_indices.push_back(ncount + t.nrm[j]);
            m.tri_to_material.push_back(t.effect);
        }
        auto it = g2s.find((int)g);
        const Mat4& M = L.scene[it == g2s.end() ? 0 : it->second].matrix;
        for (size_t j = 0; j + 2 < geo.pos.size(); j += 3) {
            const float v[4] = {geo.pos[j], geo.pos[j + 1], geo.pos[j + 2], 1.0f};
            float r[4];
            M.apply(v, r);
            if (first) {
                for (int k = 0; k < 3; ++k) m.scene_min[k] = m.scene_max[k] = r[k];
                first = false;
            } else {
                for (int k = 0; k < 3; ++k) {
                    m.scene_min[k] = m.scene_min[k] < r[k] ? m.scene_min[k] : r[k];
                    m.scene_max[k] = m.scene_max[k] > r[k] ? m.scene_max[k] : r[k];
                }
            }
            m.vertices.push_back(rt_float4{r[0], r[1], r[2], 1.0f});
            ++vcount;
        }
        for (size_t j = 0; j + 2 < geo.nrm.size(); j += 3) {
            const float v[4] = {geo.nrm[j], geo.nrm[j + 1], geo.nrm[j + 2], 0.0f};
            float r[4];
            M.apply(v, r);
            m.normals.push_back(rt_float4{r[0], r[1], r[2], 1.0f});
            ++ncount;
        }
    }
    // Index validation (the reference would read out of bounds)
    for (int32_t x : m.indices)
        if (x < 0 || x >= (int32_t)m.vertices.size()) { err = "vertex index out of range"; return -1; }
    for (int32_t x : m.normals_indices)
        if (x < 0 || x >= (int32_t)m.normals.size()) { err = "normal index out of range"; return -1; }
    if (m.materials.empty()) m.ensure_materials();
    for (int32_t x : m.tri_to_material)
        if (x < 0 || x >= (int32_t)m.materials.size()) { err = "material index out of range"; return -1; }
    return 0;
}

// Writer of the subset load_dae / ColladaLoader reads: one cook-torrance effect
// per material, one geometry with POSITION / NORMAL / TEXCOORD sources and one
// <p> per triangle, one visual-scene node with an identity <matrix>.  Floats
// are printed with 9 significant digits, so they read back bit-exactly.
int save_dae(const std::string& path, const Mesh& m, std::string& err) {
    FILE* f = std::fopen(path.c_str(), "wb");
    if (!f) { err = "cannot create " + path; return -1; }
    std::vector<char> iobuf(1 << 20);
    std::setvbuf(f, iobuf.data(), _IOFBF, iobuf.size());
    auto g = [](float x) {
        char b[32];
        std::snprintf(b, sizeof b, "%.9g", (double)x);
        return std::string(b);
    };
    std::fprintf(f, "<?xml version=\"1.0\" encoding=\"utf-8\"?>\n"
                    "<COLLADA xmlns=\"http://www.collada.org/2005/11/COLLADASchema\" version=\"1.4.0\">\n"
                    "  <library_effects>\n");
    const std::vector<rt_material> mats = m.materials.empty() ? std::vector<rt_material>{default_material()} : m.materials;
    for (size_t i = 0; i < mats.size(); ++i) {
        const rt_material& t = mats[i];
        auto c4 = [&](const rt_float4& v) { return g(v.x) + " " + g(v.y) + " " + g(v.z) + " " + g(v.w); };
        std::fprintf(f, "    <effect id=\"m%zu-fx\" name=\"m%zu\">\n      <profile_COMMON>\n"
                        "        <technique sid=\"standard\">\n          <%s>\n",
                     i, i, t.technique.x == 1 ? "phong" : "cook-torrance");
        const rt_float4* col[10] = {&t.emission, &t.ambient, &t.diffuse, &t.specular, &t.shininess,
                                    &t.reflective, &t.reflectivity, &t.transparent, &t.transparency, &t.glossiness};
        for (int a = 0; a < 10; ++a) {
            const std::string v = kAttrN[a] == 4 ? c4(*col[a]) : g(col[a]->x);
            std::fprintf(f, "            <%s><%s sid=\"%s\">%s</%s></%s>\n", kAttr[a], kAttrSub[a], kAttr[a], v.c_str(),
                         kAttrSub[a], kAttr[a]);
        }
        std::fprintf(f, "          </%s>\n        </technique>\n      </profile_COMMON>\n    </effect>\n",
                     t.technique.x == 1 ? "phong" : "cook-torrance");
    }
    std::fprintf(f, "  </library_effects>\n  <library_geometries>\n");
    // The reference reads only the first <polygons> of a mesh (ColladaLoader.cpp:202),
    // which carries one material: one geometry per material used.
    const size_t ntri = m.indices.size() / 3;
    std::vector<std::vector<size_t>> by_mat(mats.size());
    for (size_t t = 0; t < ntri; ++t) {
        const int32_t mi = m.tri_to_material.empty() ? 0 : m.tri_to_material[t];
        by_mat[(size_t)mi].push_back(t);
    }
    size_t gcount = 0;
    for (size_t mi = 0; mi < mats.size(); ++mi) {
        if (by_mat[mi].empty()) continue;
        // per geometry: the vertices / normals this material's triangles use, in first-use
        // order; a single-material mesh keeps its arrays as they are (exact round trip)
        std::vector<int32_t> vmap(m.vertices.size(), -1), nmap(m.normals.size(), -1);
        std::vector<int32_t> vlist, nlist;
        if (by_mat[mi].size() == ntri) {
            for (size_t k = 0; k < m.vertices.size(); ++k) { vmap[k] = (int32_t)k; vlist.push_back((int32_t)k); }
            const size_t nn_src = m.normals_indices.empty() ? m.vertices.size() : m.normals.size();
            for (size_t k = 0; k < nn_src; ++k) { nmap[k] = (int32_t)k; nlist.push_back((int32_t)k); }
        } else {
            for (size_t t : by_mat[mi])
                for (int j = 0; j < 3; ++j) {
                    const int32_t v = m.indices[3 * t + j];
                    if (vmap[v] < 0) { vmap[v] = (int32_t)vlist.size(); vlist.push_back(v); }
                    const int32_t nn = m.normals_indices.empty() ? v : m.normals_indices[3 * t + j];
                    if (nmap[nn] < 0) { nmap[nn] = (int32_t)nlist.size(); nlist.push_back(nn); }
                }
        }
        const std::string id = "g" + std::to_string(gcount);
        std::fprintf(f, "    <geometry id=\"%s-lib\" name=\"%sMesh\">\n      <mesh>\n", id.c_str(), id.c_str());
        std::fprintf(f, "        <source id=\"%s-lib-Position\">\n          <float_array id=\"%s-lib-Position-array\" "
                        "count=\"%zu\">", id.c_str(), id.c_str(), vlist.size() * 3);
        for (size_t k = 0; k < vlist.size(); ++k) {
            const rt_float4& v = m.vertices[vlist[k]];
            std::fprintf(f, "%s%s %s %s", k ? " " : "", g(v.x).c_str(), g(v.y).c_str(), g(v.z).c_str());
        }
        std::fprintf(f, "</float_array>\n        </source>\n");
        std::fprintf(f, "        <source id=\"%s-lib-Normal0\">\n          <float_array id=\"%s-lib-Normal0-array\" "
                        "count=\"%zu\">", id.c_str(), id.c_str(), nlist.size() * 3);
        for (size_t k = 0; k < nlist.size(); ++k) {
            const rt_float4& v = m.normals[nlist[k]];
            std::fprintf(f, "%s%s %s %s", k ? " " : "", g(v.x).c_str(), g(v.y).c_str(), g(v.z).c_str());
        }
        std::fprintf(f, "</float_array>\n        </source>\n");
        std::fprintf(f, "        <source id=\"%s-lib-UV0\">\n          <float_array id=\"%s-lib-UV0-array\" "
                        "count=\"2\">0 0</float_array>\n        </source>\n", id.c_str(), id.c_str());
        std::fprintf(f, "        <vertices id=\"%s-lib-Vertex\">\n          <input semantic=\"POSITION\" "
                        "source=\"#%s-lib-Position\"/>\n        </vertices>\n", id.c_str(), id.c_str());
        std::fprintf(f, "        <polygons material=\"m%zu\" count=\"%zu\">\n"
                        "          <input semantic=\"VERTEX\" offset=\"0\" source=\"#%s-lib-Vertex\"/>\n"
                        "          <input semantic=\"NORMAL\" offset=\"1\" source=\"#%s-lib-Normal0\"/>\n"
                        "          <input semantic=\"TEXCOORD\" offset=\"2\" set=\"0\" source=\"#%s-lib-UV0\"/>\n",
                     mi, by_mat[mi].size(), id.c_str(), id.c_str(), id.c_str());
        for (size_t t : by_mat[mi]) {
            int32_t v[3], nn[3];
            for (int j = 0; j < 3; ++j) {
                v[j] = vmap[m.indices[3 * t + j]];
                nn[j] = nmap[m.normals_indices.empty() ? m.indices[3 * t + j] : m.normals_indices[3 * t + j]];
            }
            std::fprintf(f, "          <p>%d %d 0 %d %d 0 %d %d 0</p>\n", v[0], nn[0], v[1], nn[1], v[2], nn[2]);
        }
        std::fprintf(f, "        </polygons>\n      </mesh>\n    </geometry>\n");
        ++gcount;
    }
    std::fprintf(f, "  </library_geometries>\n  <library_visual_scenes>\n    <visual_scene id=\"scene\">\n");
    for (size_t k = 0; k < gcount; ++k)
        std::fprintf(f, "      <node id=\"n%zu\" name=\"n%zu\">\n        <matrix>1 0 0 0 0 1 0 0 0 0 1 0 0 0 0 1</matrix>\n"
                        "        <instance_geometry url=\"#g%zu-lib\"/>\n      </node>\n", k, k, k);
    std::fprintf(f, "    </visual_scene>\n  </library_visual_scenes>\n</COLLADA>\n");
    const bool ok = std::ferror(f) == 0;
    std::fclose(f);
    if (!ok) { err = "write failed: " + path; return -1; }
    return 0;
}

}  // namespace rtamd
