// sp_scene.cpp -- scene description (.sp) parser, mesh readers and host math.
//
// Behavioural mirror of base/FileParser.cpp (four ordered passes, per-type attribute bodies),
// base/PlyReader.cpp:326 read_ply (vertex normals from normalised face normals),
// base/STLReader.cpp (binary STL with vertex welding), shapes/Triangle.h:25 Mesh (world-space
// pre-transform), math/Transformation.h (forward/inverse composition) and
// Cameras/Camera.h:99 PerspectiveCamera::create_transform.
#include "sp_host.hpp"

#include <algorithm>
#include <cctype>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <map>
#include <set>
#include <sstream>
#include <unordered_map>

namespace sph {

using namespace spm;

// ================================================================ linear algebra (host)
aff aff_identity()
{
    aff a;
    a.vx = mk(1, 0, 0); a.vy = mk(0, 1, 0); a.vz = mk(0, 0, 1); a.p = mk(0, 0, 0);
    return a;
}
lin lin_identity()
{
    lin l;
    l.vx = mk(1, 0, 0); l.vy = mk(0, 1, 0); l.vz = mk(0, 0, 1);
    return l;
}
// LinearSpace3x3 * Vector3 (math/LinearSpace3x3.h:220): madd(b.x, c0, madd(b.y, c1, b.z * c2))
static f3 lin_apply(const f3& c0, const f3& c1, const f3& c2, f3 b) { return xfm_vector(c0, c1, c2, b); }
lin lin_mul(const lin& a, const lin& b)
{
    lin r;
    r.vx = lin_apply(a.vx, a.vy, a.vz, b.vx);
    r.vy = lin_apply(a.vx, a.vy, a.vz, b.vy);
    r.vz = lin_apply(a.vx, a.vy, a.vz, b.vz);
    return r;
}
// AffineSpace * AffineSpace (math/AffineSpace.h:170): {a.l*b.l, a.l*b.p + a.p}
aff aff_mul(const aff& a, const aff& b)
{
    lin al{ a.vx, a.vy, a.vz }, bl{ b.vx, b.vy, b.vz };
    lin l = lin_mul(al, bl);
    aff r;
    r.vx = l.vx; r.vy = l.vy; r.vz = l.vz;
    r.p  = add(lin_apply(a.vx, a.vy, a.vz, b.p), a.p);
    return r;
}
// AffineSpace * LinearSpace3x3 (math/AffineSpace.h:175): {a.l*b, a.p}
aff aff_mul_lin(const aff& a, const lin& b)
{
    lin al{ a.vx, a.vy, a.vz };
    lin l = lin_mul(al, b);
    aff r;
    r.vx = l.vx; r.vy = l.vy; r.vz = l.vz; r.p = a.p;
    return r;
}
// LinearSpace3x3 * AffineSpace (math/AffineSpace.h:182): {a*b.l, a*b.p}
aff lin_mul_aff(const lin& a, const aff& b)
{
    lin bl{ b.vx, b.vy, b.vz };
    lin l = lin_mul(a, bl);
    aff r;
    r.vx = l.vx; r.vy = l.vy; r.vz = l.vz;
    r.p  = lin_apply(a.vx, a.vy, a.vz, b.p);
    return r;
}
lin lin_transposed(const lin& a)
{
    lin r;
    r.vx = mk(a.vx.x, a.vy.x, a.vz.x);
    r.vy = mk(a.vx.y, a.vy.y, a.vz.y);
    r.vz = mk(a.vx.z, a.vy.z, a.vz.z);
    return r;
}
// LinearSpace3x3::inverse (math/LinearSpace3x3.h:277): adjoint() / determinant()
lin lin_inverse(const lin& a)
{
    lin adj{ cross(a.vy, a.vz), cross(a.vz, a.vx), cross(a.vx, a.vy) };
    adj             = lin_transposed(adj);
    const float det = dot(a.vx, cross(a.vy, a.vz));
    lin r;
    r.vx = divs(adj.vx, det);
    r.vy = divs(adj.vy, det);
    r.vz = divs(adj.vz, det);
    return r;
}
lin normal_matrix(const aff& m)
{
    lin l{ m.vx, m.vy, m.vz };
    return lin_transposed(lin_inverse(l));
}
f3 xfm_normal(const lin& nm, f3 n) { return xfm_vector(nm, n); }

// ---- Transformation factories (math/Transformation.h:122-142)
static lin lin_scale(f3 s)
{
    lin l;
    l.vx = mk(s.x, 0, 0); l.vy = mk(0, s.y, 0); l.vz = mk(0, 0, s.z);
    return l;
}
static lin lin_rotate(f3 u, float radians)
{
    // LinearSpace3x3::rotate (math/LinearSpace3x3.h:132); row-major constructor -> columns
    u             = host_normalize(u);
    const float s = std::sin(radians);
    const float c = std::cos(radians);
    const float m00 = u.x * u.x + (1 - u.x * u.x) * c;
    const float m01 = u.x * u.y * (1 - c) - u.z * s;
    const float m02 = u.x * u.z * (1 - c) + u.y * s;
    const float m10 = u.x * u.y * (1 - c) + u.z * s;
    const float m11 = u.y * u.y + (1 - u.y * u.y) * c;
    const float m12 = u.y * u.z * (1 - c) - u.x * s;
    const float m20 = u.x * u.z * (1 - c) - u.y * s;
    const float m21 = u.y * u.z * (1 - c) + u.x * s;
    const float m22 = u.z * u.z + (1 - u.z * u.z) * c;
    lin l;
    l.vx = mk(m00, m10, m20);
    l.vy = mk(m01, m11, m21);
    l.vz = mk(m02, m12, m22);
    return l;
}
static float degrees_to_radians(float deg) { return deg * k_pi / 180.0f; } // math/Angles.h:122

static void append_translate(AffXf& t, f3 p)
{
    aff f = aff_identity(); f.p = p;
    aff i = aff_identity(); i.p = neg(p);
    t.fwd = aff_mul(t.fwd, f);
    t.inv = aff_mul(i, t.inv);
}
static void append_linear(AffXf& t, const lin& f, const lin& i)
{
    t.fwd = aff_mul_lin(t.fwd, f);
    t.inv = lin_mul_aff(i, t.inv);
}
static void append_rotate(AffXf& t, f3 axis, float deg)
{
    const float r = degrees_to_radians(deg);
    append_linear(t, lin_rotate(axis, r), lin_rotate(axis, -r));
}
static void append_scale(AffXf& t, f3 s)
{
    if (s.x == 0.0f || s.y == 0.0f || s.z == 0.0f) throw SpError(SP_ERR_PARSE, "Unable to handle zero scale");
    append_linear(t, lin_scale(s), lin_scale(mk(1.0f / s.x, 1.0f / s.y, 1.0f / s.z)));
}

// ================================================================ camera
aff perspective_camera_transform(f3 eye, f3 look_at, f3 up, float fov_degrees, int w, int h)
{
    const float fov_scale = 1.0f / std::tan(0.5f * degrees_to_radians(fov_degrees));
    // AffineSpace::look_at (math/AffineSpace.h:59)
    const f3 z = host_normalize(sub(look_at, eye));
    const f3 u = host_normalize(cross(up, z));
    const f3 v = host_normalize(cross(z, u));
    const f3 vx = u;
    const f3 vy = neg(v);
    const f3 t0 = scale(-0.5f * (float)w, u);
    const f3 t1 = scale(0.5f * (float)h, v);
    const f3 t2 = scale(0.5f * (float)h * fov_scale, z);
    const f3 vz = add(add(t0, t1), t2);
    aff a;
    a.vx = vx; a.vy = vy; a.vz = vz; a.p = eye;
    return a;
}

void Scene::rebuild_camera()
{
    camera = perspective_camera_transform(cam_origin, cam_look_at, cam_up, cam_fov_deg, image_width, image_height);
}

void rsequence_alphas(float alpha1[1], float alpha2[2])
{
    auto phi = [](unsigned dim) {
        float x = 2.0f;
        for (int i = 0; i < 10; ++i) x = std::pow(1.0f + x, 1.0f / (static_cast<float>(dim) + 1.0f));
        return x;
    };
    auto mod1 = [](float f) { float d; return std::modf(f, &d); };
    const float g1 = phi(1), g2 = phi(2);
    alpha1[0] = mod1(std::pow(1.0f / g1, 0u + 1.0f));
    alpha2[0] = mod1(std::pow(1.0f / g2, 0u + 1.0f));
    alpha2[1] = mod1(std::pow(1.0f / g2, 1u + 1.0f));
}

// ================================================================ text stream (istream-like)
namespace {
struct Cursor {
    const std::string& s;
    size_t             pos = 0;
    bool               fail = false;
    explicit Cursor(const std::string& str) : s(str) {}
    bool eof() const { return pos >= s.size(); }
    void skip_ws()
    {
        while (pos < s.size() && std::isspace(static_cast<unsigned char>(s[pos]))) ++pos;
    }
    // Token >> (base/FileParser.cpp:123): whitespace then [A-Za-z0-9_]*
    std::string token()
    {
        skip_ws();
        std::string t;
        while (pos < s.size() && (s[pos] == '_' || std::isalnum(static_cast<unsigned char>(s[pos])))) t.push_back(s[pos++]);
        return t;
    }
    char get_char()
    {
        skip_ws();
        if (pos >= s.size()) { fail = true; return 0; }
        return s[pos++];
    }
    float get_float()
    {
        skip_ws();
        if (fail || pos >= s.size()) { fail = true; return 0.0f; }
        const char* b = s.c_str() + pos;
        char*       e = nullptr;
        const float v = std::strtof(b, &e);
        if (e == b) { fail = true; return 0.0f; }
        pos += static_cast<size_t>(e - b);
        return v;
    }
    int get_int()
    {
        skip_ws();
        if (fail || pos >= s.size()) { fail = true; return 0; }
        const char* b = s.c_str() + pos;
        char*       e = nullptr;
        const long  v = std::strtol(b, &e, 10);
        if (e == b) { fail = true; return 0; }
        pos += static_cast<size_t>(e - b);
        return static_cast<int>(v);
    }
    std::string get_word()
    {
        skip_ws();
        std::string w;
        while (pos < s.size() && !std::isspace(static_cast<unsigned char>(s[pos]))) w.push_back(s[pos++]);
        if (w.empty()) fail = true;
        return w;
    }
    // std::filesystem::path >> uses std::quoted
    std::string get_path()
    {
        skip_ws();
        if (pos < s.size() && s[pos] == '"') {
            ++pos;
            std::string w;
            while (pos < s.size() && s[pos] != '"') {
                if (s[pos] == '\\' && pos + 1 < s.size()) ++pos;
                w.push_back(s[pos++]);
            }
            if (pos < s.size()) ++pos;
            return w;
        }
        return get_word();
    }
    f3 get_vec3()
    {
        const float x = get_float(), y = get_float(), z = get_float();
        return mk(x, y, z);
    }
};

std::string trim_ws(const std::string& s)
{
    size_t b = 0, e = s.size();
    while (b < e && std::isspace(static_cast<unsigned char>(s[b]))) ++b;
    while (e > b && std::isspace(static_cast<unsigned char>(s[e - 1]))) --e;
    return s.substr(b, e - b);
}
std::string trim_char(const std::string& s, char c)
{
    size_t b = 0, e = s.size();
    while (b < e && s[b] == c) ++b;
    while (e > b && s[e - 1] == c) --e;
    return s.substr(b, e - b);
}

[[noreturn]] void parse_error(const std::string& m) { throw SpError(SP_ERR_PARSE, m); }

// ---------------------------------------------------------------- PLY
enum class PlyType { I8, U8, I16, U16, I32, U32, F32, F64, NONE };
PlyType ply_type(const std::string& s)
{
    if (s == "char" || s == "int8") return PlyType::I8;
    if (s == "uchar" || s == "uint8") return PlyType::U8;
    if (s == "short" || s == "int16") return PlyType::I16;
    if (s == "ushort" || s == "uint16") return PlyType::U16;
    if (s == "int" || s == "int32") return PlyType::I32;
    if (s == "uint" || s == "uint32") return PlyType::U32;
    if (s == "float" || s == "float32") return PlyType::F32;
    if (s == "double" || s == "float64") return PlyType::F64;
    throw SpError(SP_ERR_PARSE, "Unknown data type");
}
size_t ply_size(PlyType t)
{
    switch (t) {
    case PlyType::I8: case PlyType::U8: return 1;
    case PlyType::I16: case PlyType::U16: return 2;
    case PlyType::I32: case PlyType::U32: case PlyType::F32: return 4;
    case PlyType::F64: return 8;
    default: return 0;
    }
}

struct PlyIn {
    const std::vector<char>& buf;
    size_t                   pos;
    int                      mode; // 0 ascii, 1 LE, 2 BE
    double read(PlyType t)
    {
        if (mode == 0) {
            while (pos < buf.size() && std::isspace(static_cast<unsigned char>(buf[pos]))) ++pos;
            const char* b = buf.data() + pos;
            char*       e = nullptr;
            const double v = std::strtod(b, &e);
            pos += static_cast<size_t>(e - b);
            return v;
        }
        const size_t n = ply_size(t);
        if (pos + n > buf.size()) throw SpError(SP_ERR_IO, "Truncated PLY");
        unsigned char bytes[8];
        std::memcpy(bytes, buf.data() + pos, n);
        pos += n;
        if (mode == 2) std::reverse(bytes, bytes + n);
        switch (t) {
        case PlyType::I8: { int8_t v; std::memcpy(&v, bytes, 1); return v; }
        case PlyType::U8: { uint8_t v; std::memcpy(&v, bytes, 1); return v; }
        case PlyType::I16: { int16_t v; std::memcpy(&v, bytes, 2); return v; }
        case PlyType::U16: { uint16_t v; std::memcpy(&v, bytes, 2); return v; }
        case PlyType::I32: { int32_t v; std::memcpy(&v, bytes, 4); return v; }
        case PlyType::U32: { uint32_t v; std::memcpy(&v, bytes, 4); return v; }
        case PlyType::F32: { float v; std::memcpy(&v, bytes, 4); return v; }
        case PlyType::F64: { double v; std::memcpy(&v, bytes, 8); return v; }
        default: return 0;
        }
    }
};

std::vector<char> read_file(const std::string& path)
{
    std::ifstream in(path, std::ios::binary);
    if (!in) throw SpError(SP_ERR_IO, "File " + path + " does not exit");
    return std::vector<char>((std::istreambuf_iterator<char>(in)), std::istreambuf_iterator<char>());
}

// Vertex normals from normalised face normals (base/PlyReader.cpp:493-528).
void finish_normals(const std::vector<f3>& verts, const std::vector<std::array<uint32_t, 3>>& faces,
                    const std::vector<f3>& face_normals, std::vector<f3>& vnormals)
{
    vnormals.assign(verts.size(), mk(0, 0, 0));
    for (size_t f = 0; f < faces.size(); ++f)
        for (int i = 0; i < 3; ++i) vnormals.at(faces[f][i]) = add(vnormals.at(faces[f][i]), face_normals[f]);
    for (auto& n : vnormals) {
        // `n != Normal3{0}` uses cmpneq: true if any lane differs (NaN included)
        const bool nz = (n.x != 0.0f) || (n.y != 0.0f) || (n.z != 0.0f);
        n = nz ? host_normalize(n) : mk(0.0f, 1.0f, 0.0f);
    }
}

Mesh make_mesh(std::vector<f3> verts, std::vector<f3> normals, std::vector<uint32_t> idx, const AffXf& xf)
{
    // Mesh ctor (shapes/Triangle.h:25): transform vertices (point) and normals (inverse transpose)
    const lin nm = normal_matrix(xf.fwd);
    for (auto& v : verts) v = xfm_point(xf.fwd, v);
    for (auto& n : normals) n = xfm_normal(nm, n);
    Mesh m;
    m.vertices = std::move(verts);
    m.normals  = std::move(normals);
    m.indices  = std::move(idx);
    return m;
}

Mesh read_ply(const std::string& path, const AffXf& xf)
{
    const std::vector<char> buf = read_file(path);
    size_t                  pos = 0;
    auto next_line = [&]() -> std::string {
        while (pos < buf.size()) {
            size_t e = pos;
            while (e < buf.size() && buf[e] != '\n') ++e;
            std::string line(buf.data() + pos, buf.data() + e);
            pos = (e < buf.size()) ? e + 1 : e;
            line = trim_ws(line);
            if (line.empty() || line.rfind("comment", 0) == 0) continue;
            return line;
        }
        return std::string{};
    };
    if (next_line() != "ply") throw SpError(SP_ERR_PARSE, "Invalid PLY header");
    const std::string format = next_line();
    int mode;
    if (format == "format ascii 1.0") mode = 0;
    else if (format == "format binary_little_endian 1.0") mode = 1;
    else if (format == "format binary_big_endian 1.0") mode = 2;
    else throw SpError(SP_ERR_PARSE, "Invalid PLY format");

    uint32_t num_vertices = 0, num_faces = 0;
    std::vector<std::pair<PlyType, std::string>> vprops;
    PlyType count_t = PlyType::NONE, index_t = PlyType::NONE;
    std::string line = next_line();
    while (!line.empty() && line != "end_header") {
        if (line.rfind("element", 0) == 0) {
            std::istringstream ls(line);
            std::string kw, name, num;
            ls >> kw >> name >> num;
            if (num.empty()) throw SpError(SP_ERR_PARSE, "Unexpected argument count to 'element'");
            if (name == "vertex") {
                num_vertices = static_cast<uint32_t>(std::stoul(num));
                line         = next_line();
                while (line.rfind("property", 0) == 0) {
                    std::istringstream ps(line);
                    std::vector<std::string> parts;
                    for (std::string w; ps >> w;) parts.push_back(w);
                    if (parts.size() == 3) vprops.emplace_back(ply_type(parts[1]), parts[2]);
                    line = next_line();
                }
                continue;
            } else if (name == "face") {
                num_faces = static_cast<uint32_t>(std::stoul(num));
                line      = next_line();
                while (line.rfind("property", 0) == 0) {
                    std::istringstream ps(line);
                    std::vector<std::string> parts;
                    for (std::string w; ps >> w;) parts.push_back(w);
                    if (parts.size() == 1) throw SpError(SP_ERR_PARSE, "Malformed face property");
                    if (parts.size() == 5 && parts[1] == "list" && (parts[4] == "vertex_indices" || parts[4] == "vertex_index")) {
                        count_t = ply_type(parts[2]);
                        index_t = ply_type(parts[3]);
                    }
                    line = next_line();
                }
                continue;
            }
        }
        line = next_line();
    }
    PlyIn in{ buf, pos, mode };
    std::vector<f3> verts;
    verts.reserve(num_vertices);
    for (uint32_t i = 0; i < num_vertices; ++i) {
        float x = 0, y = 0, z = 0;
        for (auto& p : vprops) {
            const float v = static_cast<float>(in.read(p.first));
            if (p.second == "x") x = v;
            else if (p.second == "y") y = v;
            else if (p.second == "z") z = v;
        }
        verts.push_back(mk(x, y, z));
    }
    std::vector<uint32_t>                 indices;
    std::vector<std::array<uint32_t, 3>>  faces;
    std::vector<f3>                       fnormals;
    faces.reserve(num_faces);
    for (uint32_t i = 0; i < num_faces; ++i) {
        const uint64_t cnt = static_cast<uint64_t>(in.read(count_t));
        if (cnt != 3) {
            for (uint64_t v = 0; v < cnt; ++v) in.read(index_t);
            continue;
        }
        std::array<uint32_t, 3> f{};
        for (int v = 0; v < 3; ++v) f[v] = static_cast<uint32_t>(in.read(index_t));
        const f3 e0 = sub(verts.at(f[1]), verts.at(f[0]));
        const f3 e1 = sub(verts.at(f[2]), verts.at(f[0]));
        f3       fn = cross(e0, e1);
        if (dot(fn, fn) == 0.0f) continue; // zero-area face skipped
        fn = host_normalize(fn);
        for (int v = 0; v < 3; ++v) indices.push_back(f[v]);
        faces.push_back(f);
        fnormals.push_back(fn);
    }
    std::vector<f3> vnormals;
    finish_normals(verts, faces, fnormals, vnormals);
    return make_mesh(std::move(verts), std::move(vnormals), std::move(indices), xf);
}

Mesh read_stl(const std::string& path, const AffXf& xf)
{
    const std::vector<char> buf = read_file(path);
    if (buf.size() >= 5 && std::strncmp(buf.data(), "solid", 5) == 0)
        throw SpError(SP_ERR_UNSUPPORTED, "ASCII STL not implemented (base/STLReader.cpp:41)");
    if (buf.size() < 84) throw SpError(SP_ERR_IO, "Truncated STL");
    uint32_t ntri;
    std::memcpy(&ntri, buf.data() + 80, 4);
    size_t pos = 84;
    // VertexIndexer: std::map<Point3, index> keyed by <=> (x, then y, then z)
    auto less3 = [](const f3& a, const f3& b) {
        if (a.x != b.x) return a.x < b.x;
        if (a.y != b.y) return a.y < b.y;
        return a.z < b.z;
    };
    std::map<f3, uint32_t, decltype(less3)> welded(less3);
    std::vector<f3>                      verts;
    std::vector<uint32_t>                indices;
    std::vector<std::array<uint32_t, 3>> faces;
    std::vector<f3>                      fnormals;
    auto rf = [&](float& v) {
        if (pos + 4 > buf.size()) throw SpError(SP_ERR_IO, "Truncated STL");
        std::memcpy(&v, buf.data() + pos, 4);
        pos += 4;
    };
    for (uint32_t t = 0; t < ntri; ++t) {
        float nx, ny, nz;
        rf(nx); rf(ny); rf(nz);
        std::array<uint32_t, 3> f{};
        for (int j = 0; j < 3; ++j) {
            float x, y, z;
            rf(x); rf(y); rf(z);
            const f3 v  = mk(x, y, z);
            auto     it = welded.find(v);
            uint32_t id;
            if (it != welded.end()) id = it->second;
            else { id = static_cast<uint32_t>(welded.size()); welded.emplace(v, id); }
            if (id >= verts.size()) verts.push_back(v);
            f[j] = id;
            indices.push_back(id); // pushed before the zero-area check, as the reference does
        }
        pos += 2;
        f3 fn = mk(nx, ny, nz);
        auto is_zero = [](f3 a) {
            auto fc = [](float p, float q) {
                const float eps = 1.0e-05f;
                if (std::abs(p - q) <= eps) return true;
                return std::abs(p - q) <= eps * std::max(std::abs(p), std::abs(q));
            };
            return fc(a.x, 0.0f) && fc(a.y, 0.0f) && fc(a.z, 0.0f);
        };
        if (is_zero(fn)) fn = cross(sub(verts.at(f[1]), verts.at(f[0])), sub(verts.at(f[2]), verts.at(f[0])));
        if (is_zero(fn)) continue;
        fn = host_normalize(fn);
        faces.push_back(f);
        fnormals.push_back(fn);
    }
    std::vector<f3> vnormals;
    finish_normals(verts, faces, fnormals, vnormals);
    return make_mesh(std::move(verts), std::move(vnormals), std::move(indices), xf);
}

std::string ext_of(const std::string& p)
{
    const size_t slash = p.find_last_of('/');
    const size_t dot   = p.find_last_of('.');
    if (dot == std::string::npos || (slash != std::string::npos && dot < slash)) return "";
    return p.substr(dot);
}

std::string resolve(const std::string& base_dir, const std::string& p)
{
    if (p.empty() || p[0] == '/') return p;
    if (!base_dir.empty()) {
        const std::string cand = base_dir + "/" + p;
        std::ifstream     t(cand, std::ios::binary);
        if (t) return cand;
    }
    return p;
}

// file_to_string (base/FileParser.cpp:821): strip blank/comment lines and trailing comments;
// `lines` gets the 1-based source line of every kept character (the reference's line_numbers,
// which its ParsingException messages quote as " on line N")
std::string clean_text(const std::string& text, std::vector<int>& lines)
{
    std::string        out;
    std::istringstream in(text);
    int                line_no = 0;
    lines.clear();
    for (std::string line; std::getline(in, line);) {
        ++line_no;
        std::string t = trim_ws(line);
        if (t.empty() || t[0] == '#') continue;
        const size_t h = t.find('#');
        if (h != std::string::npos) t = t.substr(0, h);
        out += t;
        out.push_back(' ');
        lines.insert(lines.end(), t.size() + 1, line_no);
    }
    return out;
}

class Parser {
public:
    Parser(std::string base_dir) : m_base(std::move(base_dir)), m_scene(new Scene) {}

    std::unique_ptr<Scene> parse(const std::string& text)
    {
        const std::string clean = clean_text(text, m_lines);
        Cursor            c(clean);
        if (c.token() != "version") parse_error("Expects version as first directive");
        if (c.get_char() != ':') parse_error("Expected ':' character");
        const int version = c.get_int();
        if (version != 1) parse_error("Unable to parse version " + std::to_string(version));
        const size_t post_version = c.pos;

        static const std::set<std::string> valid = { "environment_light", "instance", "material_clearcoat",
                                                     "material_glossy", "material_lambertian",
                                                     "material_transmissive_dielectric", "mesh",
                                                     "perspective_camera", "plane", "scene_parameters",
                                                     "sphere", "sphere_light" };
        // first pass: validate types
        collect(clean, post_version, [&](const std::string& w, const std::string&) {
            if (!valid.count(w)) parse_error(on_line("Unknown type '" + w + "'", m_body_off));
        });
        run_pass(clean, post_version, { "scene_parameters" });
        run_pass(clean, post_version, { "environment_light", "material_glossy", "material_lambertian",
                                        "material_transmissive_dielectric", "perspective_camera", "sphere_light" });
        run_pass(clean, post_version, { "material_clearcoat" });
        run_pass(clean, post_version, { "instance", "mesh", "plane", "sphere" });
        if (!m_scene->has_camera) parse_error("Scene has no perspective_camera");
        return std::move(m_scene);
    }

private:
    template <typename F>
    void collect(const std::string& clean, size_t start, F fn)
    {
        Cursor c(clean);
        c.pos = start;
        while (true) {
            const std::string w = c.token();
            const size_t at = c.pos; // tellg() right after the token, before `>> c` skips blanks
            c.skip_ws();
            if (c.eof()) break;
            if (c.get_char() != '{') parse_error(on_line("Expected '{' character", at));
            const size_t close = clean.find('}', c.pos);
            const std::string body = clean.substr(c.pos, close == std::string::npos ? std::string::npos : close - c.pos);
            m_body_off = c.pos;
            c.pos = (close == std::string::npos) ? clean.size() : close + 1;
            fn(w, body);
        }
    }
    void run_pass(const std::string& clean, size_t start, const std::set<std::string>& types)
    {
        collect(clean, start, [&](const std::string& w, const std::string& body) {
            if (!types.count(w)) return;
            if (w == "scene_parameters") scene_parameters(body);
            else if (w == "environment_light") environment_light(body);
            else if (w == "material_glossy") material_glossy(body);
            else if (w == "material_lambertian") material_lambertian(body);
            else if (w == "material_clearcoat") material_clearcoat(body);
            else if (w == "perspective_camera") perspective_camera(body);
            else if (w == "sphere_light") sphere_light(body);
            else if (w == "mesh") mesh(body);
            else if (w == "plane") shape(body, SP_PRIM_PLANE);
            else if (w == "sphere") shape(body, SP_PRIM_SPHERE);
            // "instance" and "material_transmissive_dielectric" are warnings in the reference
        });
    }

    template <typename F>
    void attributes(const std::string& body, const char* what, F fn)
    {
        const size_t body_off = m_body_off;
        Cursor       c(body);
        while (true) {
            const std::string w = c.token();
            const size_t at = body_off + c.pos; // consume_character's line: tellg() before `>> c`
            c.skip_ws();
            if (c.eof() || c.fail) break;
            if (c.get_char() != ':') parse_error(on_line("Expected ':' character", at));
            if (!fn(w, c)) parse_error(on_line(std::string("Unknown ") + what + " attribute: " + w, body_off + c.pos));
            if (c.fail) break; // a failed extraction stops the reference's loop as well
        }
    }

    // m_materials.find + LOG_ERROR (base/FileParser.cpp:494-498, 555-559, 660-665): an unknown name
    // is reported and parsing goes on with the block's material left as it was (-1 on a miss), so an
    // earlier valid name stays; the block's own check ("needs a base material" / "needs a
    // material") fails only when none was found
    int find_material(const std::string& name)
    {
        for (size_t i = 0; i < m_scene->material_names.size(); ++i)
            if (m_scene->material_names[i] == name) return static_cast<int>(i);
        std::fprintf(stderr, "Material '%s' not found\n", name.c_str());
        return -1;
    }
    // the checks after a block's attribute loop (base/FileParser.cpp:408-416): the loop only ends
    // with the stream failed, so tellg() is -1 and the line is that of offset-1, the block's '{'
    std::string at_block_end(const std::string& what) const { return on_line(what, m_body_off - 1); }
    void add_material(const std::string& name, const sp_material_desc& d)
    {
        if (name.empty()) parse_error(at_block_end("Material needs named"));
        for (auto& n : m_scene->material_names)
            if (n == name) parse_error(at_block_end("Material " + name + " already exists"));
        m_scene->material_names.push_back(name);
        m_scene->materials.push_back(Material{ d });
    }
    static sp_material_desc blank_material()
    {
        sp_material_desc d{};
        d.base = -1;
        d.sample_visible_area = 1;
        return d;
    }

    void scene_parameters(const std::string& body)
    {
        attributes(body, "scene_parameters", [&](const std::string& w, Cursor& c) {
            if (w == "output_file_name") m_scene->output_file_name = trim_char(c.get_word(), '"');
            else if (w == "width") m_scene->image_width = c.get_int();
            else if (w == "height") m_scene->image_height = c.get_int();
            else if (w == "russian_roulette_depth") m_scene->rr_depth = c.get_int();
            else if (w == "max_depth") m_scene->max_depth = c.get_int();
            else if (w == "integrator") {
                int32_t t;
                if (sp_string_to_integrator(c.get_word().c_str(), &t) != SP_OK) parse_error("Unknown integrator type");
                m_scene->integrator = t;
            } else return false;
            return true;
        });
    }
    // FileParser::parse_environment_light (base/FileParser.cpp:325)
    void environment_light(const std::string& body)
    {
        rgb         radiance = mkc(1, 1, 1);
        std::string image;
        float       max_radiance = 3.40282347e38f; // std::numeric_limits<float>::max()
        AffXf       xf{ aff_identity(), aff_identity() }; // LinearTransformation: p stays unused
        attributes(body, "environment light", [&](const std::string& w, Cursor& c) {
            if (w == "radiance") { f3 v = c.get_vec3(); radiance = mkc(v.x, v.y, v.z); }
            else if (w == "max_radiance") max_radiance = c.get_float();
            else if (w == "image") image = c.get_path();
            else if (w == "rotate") { f3 a = c.get_vec3(); float d = c.get_float(); append_rotate(xf, a, d); }
            else if (w == "scale") append_scale(xf, c.get_vec3());
            else return false;
            return true;
        });
        sp_light_desc l{};
        l.image       = -1;
        l.radiance[0] = radiance.r; l.radiance[1] = radiance.g; l.radiance[2] = radiance.b;
        if (image.empty()) {
            l.kind = SP_LIGHT_ENVIRONMENT;
        } else {
            // `read(filename)` then `img *= radiance` (FileParser.cpp:366-367).  The reference
            // resolves the path against the working directory; here the scene file's directory
            // is tried first (resolve()).
            EnvImage e;
            read_pfm(resolve(m_base, image), e.width, e.height, e.pixels);
            for (size_t i = 0; i < e.pixels.size(); i += 3) {
                e.pixels[i] *= radiance.r;
                e.pixels[i + 1] *= radiance.g;
                e.pixels[i + 2] *= radiance.b;
            }
            e.max_radiance   = max_radiance;
            e.light_to_world = lin{ xf.fwd.vx, xf.fwd.vy, xf.fwd.vz };
            e.world_to_light = lin{ xf.inv.vx, xf.inv.vy, xf.inv.vz };
            l.kind  = SP_LIGHT_IMAGE_ENVIRONMENT;
            l.image = (int32_t)m_scene->env_images.size();
            m_scene->env_images.push_back(std::move(e));
        }
        m_scene->lights.push_back(l);
    }
    void material_lambertian(const std::string& body)
    {
        std::string name;
        rgb         albedo = mkc(0, 0, 0);
        attributes(body, "material_lambertian", [&](const std::string& w, Cursor& c) {
            if (w == "name") name = trim_char(c.get_word(), '"');
            else if (w == "diffuse") { f3 v = c.get_vec3(); albedo = mkc(v.x, v.y, v.z); }
            else return false;
            return true;
        });
        sp_material_desc d = blank_material();
        d.kind             = SP_MAT_LAMBERTIAN;
        const rgb a        = cdivs(albedo, k_pi); // LambertianBRDF ctor
        d.lambert_albedo[0] = a.r; d.lambert_albedo[1] = a.g; d.lambert_albedo[2] = a.b;
        add_material(name, d);
    }
    static float roughness_to_alpha(float roughness)
    {
        roughness     = std_max(roughness, 1e-3f);
        const float x = std::log(roughness);
        return 1.62142f + 0.819955f * x + 0.1734f * x * x + 0.0171201f * x * x * x + 0.000640711f * x * x * x * x;
    }
    void material_glossy(const std::string& body)
    {
        std::string name;
        rgb         color     = mkc(0, 0, 0);
        float       roughness = 0.5f, ior = 1.5f;
        attributes(body, "material_glossy", [&](const std::string& w, Cursor& c) {
            if (w == "name") name = trim_char(c.get_word(), '"');
            else if (w == "diffuse") { f3 v = c.get_vec3(); color = mkc(v.x, v.y, v.z); }
            else if (w == "roughness") roughness = c.get_float();
            else if (w == "ior") ior = c.get_float();
            else return false;
            return true;
        });
        sp_material_desc d = blank_material();
        d.kind             = SP_MAT_GLOSSY;
        d.microfacet_r[0] = d.microfacet_r[1] = d.microfacet_r[2] = 1.0f;
        d.alpha_x = d.alpha_y = roughness_to_alpha(roughness);
        d.microfacet_ior      = ior;
        const rgb a           = cdivs(color, k_pi);
        d.lambert_albedo[0] = a.r; d.lambert_albedo[1] = a.g; d.lambert_albedo[2] = a.b;
        add_material(name, d);
    }
    void material_clearcoat(const std::string& body)
    {
        std::string name;
        int         base  = -1;
        float       ior   = 1.5f;
        rgb         color = mkc(1, 1, 1);
        attributes(body, "material_clearcoat", [&](const std::string& w, Cursor& c) {
            if (w == "name") name = trim_char(c.get_word(), '"');
            else if (w == "base") { if (const int m = find_material(trim_char(c.get_word(), '"')); m >= 0) base = m; }
            else if (w == "color") { f3 v = c.get_vec3(); color = mkc(v.x, v.y, v.z); }
            else if (w == "ior") ior = c.get_float();
            else return false;
            return true;
        });
        if (name.empty()) parse_error(at_block_end("Material needs named"));
        if (base < 0) parse_error(at_block_end("Clearcoat material needs a base material"));
        sp_material_desc d = blank_material();
        d.kind             = SP_MAT_CLEARCOAT;
        d.base             = base;
        d.coat_ior         = ior;
        d.coat_color[0] = color.r; d.coat_color[1] = color.g; d.coat_color[2] = color.b;
        add_material(name, d);
    }
    void perspective_camera(const std::string& body)
    {
        f3    origin{}, look{}, up = mk(0, 1, 0);
        float fov = 45.0f;
        attributes(body, "perspective_camera", [&](const std::string& w, Cursor& c) {
            if (w == "origin") origin = c.get_vec3();
            else if (w == "look_at") look = c.get_vec3();
            else if (w == "up") up = c.get_vec3();
            else if (w == "fov") fov = c.get_float();
            else return false;
            return true;
        });
        Scene& s      = *m_scene;
        s.cam_origin  = origin;
        s.cam_look_at = look;
        s.cam_up      = up;
        s.cam_fov_deg = fov;
        s.has_camera  = true;
        s.rebuild_camera();
    }
    void sphere_light(const std::string& body)
    {
        AffXf xf{ aff_identity(), aff_identity() };
        rgb   radiance = mkc(1, 1, 1);
        attributes(body, "environment light", [&](const std::string& w, Cursor& c) {
            if (w == "radiance") { f3 v = c.get_vec3(); radiance = mkc(v.x, v.y, v.z); }
            else if (w == "translate") append_translate(xf, c.get_vec3());
            else if (w == "rotate") { f3 a = c.get_vec3(); float d = c.get_float(); append_rotate(xf, a, d); }
            else if (w == "scale") append_scale(xf, c.get_vec3());
            else return false;
            return true;
        });
        sp_light_desc l{};
        l.kind = SP_LIGHT_SPHERE;
        l.image = -1;
        l.radiance[0] = radiance.r; l.radiance[1] = radiance.g; l.radiance[2] = radiance.b;
        to_desc(xf.fwd, l.object_to_world);
        to_desc(xf.inv, l.world_to_object);
        to_desc(normal_matrix(xf.fwd), l.normal_to_world);
        m_scene->lights.push_back(l);
    }
    void mesh(const std::string& body)
    {
        AffXf       xf{ aff_identity(), aff_identity() };
        int         material = -1;
        std::string path;
        attributes(body, "mesh", [&](const std::string& w, Cursor& c) {
            if (w == "material") { if (const int m = find_material(trim_char(c.get_word(), '"')); m >= 0) material = m; }
            else if (w == "file") path = c.get_path();
            else if (w == "translate") append_translate(xf, c.get_vec3());
            else if (w == "rotate") { f3 a = c.get_vec3(); float d = c.get_float(); append_rotate(xf, a, d); }
            else if (w == "scale") append_scale(xf, c.get_vec3());
            else return false;
            return true;
        });
        if (material < 0) parse_error("mesh needs a material");
        const std::string full = resolve(m_base, path);
        const std::string ext  = ext_of(path);
        Mesh              m;
        if (ext == ".ply") m = read_ply(full, xf);
        else if (ext == ".stl") m = read_stl(full, xf);
        else return; // LOG_ERROR + return in the reference
        Scene&         s     = *m_scene;
        const uint32_t vbase = static_cast<uint32_t>(s.vertices.size());
        s.vertices.insert(s.vertices.end(), m.vertices.begin(), m.vertices.end());
        s.normals.insert(s.normals.end(), m.normals.begin(), m.normals.end());
        const size_t ntri = m.indices.size() / 3;
        for (size_t t = 0; t < ntri; ++t) {
            const int32_t tri_id = static_cast<int32_t>(s.tri_material.size());
            for (int k = 0; k < 3; ++k) s.indices.push_back(vbase + m.indices[t * 3 + k]);
            s.tri_material.push_back(material);
            s.prim_kind.push_back(SP_PRIM_TRIANGLE);
            s.prim_index.push_back(tri_id);
        }
    }
    void shape(const std::string& body, int kind)
    {
        AffXf xf{ aff_identity(), aff_identity() };
        int   material = -1;
        attributes(body, kind == SP_PRIM_PLANE ? "plane" : "sphere", [&](const std::string& w, Cursor& c) {
            if (w == "material") { if (const int m = find_material(trim_char(c.get_word(), '"')); m >= 0) material = m; }
            else if (w == "translate") append_translate(xf, c.get_vec3());
            else if (w == "rotate") { f3 a = c.get_vec3(); float d = c.get_float(); append_rotate(xf, a, d); }
            else if (w == "scale") append_scale(xf, c.get_vec3());
            else return false;
            return true;
        });
        if (material < 0) parse_error("shape needs a material");
        sp_xform_shape sh{};
        to_desc(xf.fwd, sh.object_to_world);
        to_desc(xf.inv, sh.world_to_object);
        to_desc(normal_matrix(xf.fwd), sh.normal_to_world);
        sh.material = material;
        sh.kind     = kind;
        m_scene->prim_kind.push_back(kind);
        m_scene->prim_index.push_back(static_cast<int32_t>(m_scene->shapes.size()));
        m_scene->shapes.push_back(sh);
    }
    static void put3(float* d, f3 v) { d[0] = v.x; d[1] = v.y; d[2] = v.z; }
    static void to_desc(const aff& a, sp_affine& d) { put3(d.vx, a.vx); put3(d.vy, a.vy); put3(d.vz, a.vz); put3(d.p, a.p); }
    static void to_desc(const lin& a, sp_linear& d) { put3(d.vx, a.vx); put3(d.vy, a.vy); put3(d.vz, a.vz); }

    // ParsingException(what, line) (base/FileParser.cpp:35): "<what> on line <N>", N = the source
    // line of the cleaned-text offset the reference's stream had reached
    std::string on_line(const std::string& what, size_t off) const
    {
        if (m_lines.empty()) return what;
        return what + " on line " + std::to_string(m_lines[std::min(off, m_lines.size() - 1)]);
    }

    std::string            m_base;
    std::unique_ptr<Scene> m_scene;
    std::vector<int>       m_lines;        // clean_text line numbers
    size_t                 m_body_off = 0; // clean-text offset of the block body being parsed
};
} // namespace

std::unique_ptr<Scene> parse_scene(const std::string& text, const std::string& base_dir)
{
    Parser p(base_dir);
    return p.parse(text);
}

std::unique_ptr<Scene> parse_scene_file(const std::string& path)
{
    std::ifstream in(path);
    if (!in) throw SpError(SP_ERR_IO, "Unable to open file " + path);
    std::stringstream ss;
    ss << in.rdbuf();
    const size_t slash = path.find_last_of('/');
    return parse_scene(ss.str(), slash == std::string::npos ? std::string(".") : path.substr(0, slash));
}

} // namespace sph
