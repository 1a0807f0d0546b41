// ref_harness.cpp -- TEST INFRASTRUCTURE ONLY (never part of the product).
//
// Renders tiles with the REFERENCE's own code: the scene is assembled from the reference's
// classes (PerspectiveCamera, OneSampleMaterial / ClearcoatMaterial via create_*_material, Mesh +
// Triangle, Sphere, Plane, SphereLight, EnvironmentLight, ImageBasedEnvironmentLight with the
// reference's read_pfm, Scene with its ListAccelerator/BVH)
// and every pixel runs main.cpp's render_thread body (main.cpp:86-103) with the reference's
// samplers and Integrator.  Compiled by oracle/build_ref.sh directly from the sources under
// /root/reference into oracle/_ref/libsp_ref.so; tests/test_oracle_vs_ref.py checks the C
// oracle (oracle/sp_oracle.c) against it bit for bit.
//
// What is NOT the reference here: base/FileParser.cpp and base/PlyReader.cpp need C++23
// (std::unreachable, std::format) that this image's g++ 11 lacks, so this file restates the
// few lines of scene-file tokenising (FileParser.cpp:180-300 passes, attribute loops) and PLY
// reading (PlyReader.cpp:430-530: triangle faces, zero-area faces skipped, vertex normal =
// normalize(sum of normalized face normals)) -- using the reference's own types, operator>>,
// transform builders (translate/rotate/scale, `transform *= t`) and vector math for all
// arithmetic.  Supported: the scene blocks the benchmark/test scenes use.
#include "Cameras/Camera.h"
#include "Integrators/Integrator.h"
#include "Lights/Light.h"
#include "base/MemoryArena.h"
#include "base/Scene.h"
#include "base/Tile.h"
#include "materials/Material.h"
#include "math/Sampler.h"
#include "math/Transformation.h"
#include "shapes/Plane.h"
#include "shapes/Primitive.h"
#include "shapes/Sphere.h"
#include "shapes/Triangle.h"

#include <cstdint>
#include <cstring>
#include <filesystem>
#include <fstream>
#include <map>
#include <memory>
#include <ranges>
#include <sstream>
#include <string>
#include <thread>
#include <vector>

namespace sp {
int k_pretty_print_key = -1; // defined by main.cpp:33, the driver this harness stands in for
}

namespace {

using namespace sp;

std::string g_error;

std::string trim_quotes(std::string s)
{
    while (!s.empty() && s.front() == '"') s.erase(s.begin());
    while (!s.empty() && s.back() == '"') s.pop_back();
    return s;
}

// "key:" tokens of a block body (FileParser Token + consume_character(':'))
bool next_key(std::istream& ins, std::string& key)
{
    key.clear();
    char c;
    while (ins.get(c) && std::isspace(static_cast<unsigned char>(c))) {}
    if (!ins) return false;
    do {
        if (c == ':') return true;
        key.push_back(c);
    } while (ins.get(c));
    return false;
}

struct Block {
    std::string type, body;
};

std::vector<Block> read_blocks(const std::string& path)
{
    std::ifstream      f(path);
    std::ostringstream cleaned; // FileParser file_to_string: drop blank and '#' lines
    for (std::string line; std::getline(f, line);) {
        const auto b = line.find_first_not_of(" \t\r");
        if (b == std::string::npos || line[b] == '#') continue;
        cleaned << line << '\n';
    }
    std::istringstream ins(cleaned.str());
    std::vector<Block> out;
    std::string        word;
    while (ins >> word) {
        if (word.rfind("version", 0) == 0) { // "version: 1"
            if (word.find(':') == std::string::npos) ins >> word;
            ins >> word;
            continue;
        }
        char brace;
        ins >> brace; // '{'
        std::string body;
        std::getline(ins, body, '}');
        out.push_back({ word, body });
    }
    return out;
}

// PlyReader restatement (binary_little_endian, float vertex properties, `list uchar int` faces)
std::shared_ptr<Mesh> read_ply_mesh(const std::filesystem::path& path, const AffineTransformation& object_to_world)
{
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open " + path.string());
    std::string line;
    size_t      nv = 0, nf = 0;
    int         n_vprops = 0, xi = -1, yi = -1, zi = -1;
    bool        in_vertex = false;
    while (std::getline(f, line)) {
        std::istringstream ls(line);
        std::string        w;
        ls >> w;
        if (w == "element") {
            std::string what;
            ls >> what;
            in_vertex = what == "vertex";
            if (in_vertex) ls >> nv;
            else if (what == "face") ls >> nf;
        } else if (w == "property" && in_vertex) {
            std::string type, name;
            ls >> type >> name;
            if (type != "float") throw std::runtime_error("harness: only float vertex properties");
            if (name == "x") xi = n_vprops;
            if (name == "y") yi = n_vprops;
            if (name == "z") zi = n_vprops;
            ++n_vprops;
        } else if (w == "format" && line.find("binary_little_endian") == std::string::npos) {
            throw std::runtime_error("harness: only binary_little_endian PLY");
        } else if (w == "end_header") {
            break;
        }
    }
    std::vector<Point3> vertices;
    vertices.reserve(nv);
    std::vector<float> rec(n_vprops);
    for (size_t i = 0; i < nv; ++i) {
        f.read(reinterpret_cast<char*>(rec.data()), 4 * n_vprops);
        vertices.emplace_back(rec[xi], rec[yi], rec[zi]);
    }
    std::vector<std::size_t>              indices;
    std::vector<std::array<unsigned, 3>> faces;
    std::vector<Normal3>                  face_normals;
    for (size_t i = 0; i < nf; ++i) {
        unsigned char cnt;
        f.read(reinterpret_cast<char*>(&cnt), 1);
        std::vector<int32_t> vi(cnt);
        f.read(reinterpret_cast<char*>(vi.data()), 4 * cnt);
        if (cnt != 3) continue; // PlyReader: non-triangular faces skipped
        std::array<unsigned, 3> fv{ (unsigned)vi[0], (unsigned)vi[1], (unsigned)vi[2] };
        const Vector3 edge0 = vertices.at(fv[1]) - vertices.at(fv[0]);
        const Vector3 edge1 = vertices.at(fv[2]) - vertices.at(fv[0]);
        Normal3       fn    = Normal3{ cross(edge0, edge1) };
        if (sqr_length(fn) == 0.0f) continue; // zero-area face skipped
        fn = normalize(fn);
        for (int v = 0; v < 3; ++v) indices.push_back(fv[v]);
        faces.push_back(fv);
        face_normals.push_back(fn);
    }
    std::vector vertex_normals(nv, Normal3{ 0.0f, 0.0f, 0.0f });
    for (size_t k = 0; k < faces.size(); ++k)
        for (int i = 0; i < 3; ++i) vertex_normals.at(faces[k][i]) += face_normals[k];
    for (auto& n : vertex_normals) {
        if (n != Normal3{ 0.0f, 0.0f, 0.0f }) n = normalize(n);
        else n = Normal3{ 0.0f, 1.0f, 0.0f };
    }
    return std::make_shared<Mesh>(Mesh{ std::move(indices), std::move(vertices), std::move(vertex_normals), object_to_world });
}

// STLReader restatement (base/STLReader.cpp:46 read_binary_stl, which g++ 11 cannot compile
// here): std::map<Point3, index> vertex welding, the file's face normal unless is_zero (then the
// edge cross product), zero-area faces skipped after their indices were pushed, vertex normals
// = normalize(sum of face normals).
std::shared_ptr<Mesh> read_stl_mesh(const std::filesystem::path& path, const AffineTransformation& object_to_world)
{
    std::ifstream ins(path, std::ios::binary);
    if (!ins) throw std::runtime_error("cannot open " + path.string());
    std::array<char, 80> header;
    ins.read(header.data(), 80);
    std::uint32_t num_triangles = 0;
    ins.read(reinterpret_cast<char*>(&num_triangles), 4);
    std::map<Point3, std::size_t>        index_of;
    std::vector<Point3>                  vertices;
    std::vector<std::size_t>             vertex_indices;
    std::vector<std::array<unsigned, 3>> faces;
    std::vector<Normal3>                 face_normals;
    for (std::uint32_t i = 0; i < num_triangles; ++i) {
        float nx, ny, nz;
        ins.read(reinterpret_cast<char*>(&nx), 4);
        ins.read(reinterpret_cast<char*>(&ny), 4);
        ins.read(reinterpret_cast<char*>(&nz), 4);
        Normal3                 fn{ nx, ny, nz };
        std::array<unsigned, 3> fv{};
        for (std::size_t j = 0; j < 3; ++j) {
            float x, y, z;
            ins.read(reinterpret_cast<char*>(&x), 4);
            ins.read(reinterpret_cast<char*>(&y), 4);
            ins.read(reinterpret_cast<char*>(&z), 4);
            const Point3 v{ x, y, z };
            std::size_t  index;
            if (const auto it = index_of.find(v); it != index_of.end()) {
                index = it->second;
            } else {
                index = index_of.size();
                index_of.emplace(v, index);
            }
            if (index >= vertices.size()) vertices.push_back(v);
            fv[j] = static_cast<unsigned>(index);
            vertex_indices.push_back(index);
        }
        std::uint16_t attributes;
        ins.read(reinterpret_cast<char*>(&attributes), 2);
        if (is_zero(fn)) {
            const Vector3 edge0 = vertices.at(fv[1]) - vertices.at(fv[0]);
            const Vector3 edge1 = vertices.at(fv[2]) - vertices.at(fv[0]);
            fn                  = Normal3{ cross(edge0, edge1) };
        }
        if (is_zero(fn)) continue;
        fn = normalize(fn);
        faces.push_back(fv);
        face_normals.push_back(fn);
    }
    std::vector vertex_normals(vertices.size(), Normal3{ 0.0f, 0.0f, 0.0f });
    for (size_t k = 0; k < faces.size(); ++k)
        for (int i = 0; i < 3; ++i) vertex_normals.at(faces[k][i]) += face_normals[k];
    for (auto& n : vertex_normals) {
        if (n != Normal3{ 0.0f, 0.0f, 0.0f }) n = normalize(n);
        else n = Normal3{ 0.0f, 1.0f, 0.0f };
    }
    return std::make_shared<Mesh>(Mesh{ std::move(vertex_indices), std::move(vertices), std::move(vertex_normals), object_to_world });
}

template <typename F>
void parse_attrs(const std::string& body, F&& f)
{
    std::istringstream ins(body);
    std::string        key;
    while (next_key(ins, key)) f(key, ins);
}

struct Built {
    std::unique_ptr<Scene> scene;
};

std::unique_ptr<Scene> build_scene(const std::string& path, int width, int height)
{
    const auto blocks   = read_blocks(path);
    const auto base_dir = std::filesystem::path(path).parent_path();
    int        w = 512, h = 512, rr = 3, max_depth = 10;
    for (const auto& b : blocks) { // pass 0: scene_parameters
        if (b.type != "scene_parameters") continue;
        parse_attrs(b.body, [&](const std::string& k, std::istream& ins) {
            std::string s;
            if (k == "width") ins >> w;
            else if (k == "height") ins >> h;
            else if (k == "russian_roulette_depth") ins >> rr;
            else if (k == "max_depth") ins >> max_depth;
            else ins >> s;
        });
    }
    if (width > 0) w = width;
    if (height > 0) h = height;

    std::map<std::string, std::shared_ptr<Material>> materials;
    Scene::LightContainer                            lights;
    std::unique_ptr<Camera>                          camera;
    for (const auto& b : blocks) { // pass 1: lights, basic materials, camera (file order)
        if (b.type == "material_lambertian" || b.type == "material_glossy") {
            std::string name;
            RGB         color;
            float       roughness = 0.5f, ior = 1.5f;
            parse_attrs(b.body, [&](const std::string& k, std::istream& ins) {
                if (k == "name") { ins >> name; name = trim_quotes(name); }
                else if (k == "diffuse") ins >> color;
                else if (k == "roughness") ins >> roughness;
                else if (k == "ior") ins >> ior;
            });
            if (b.type == "material_lambertian")
                materials[name] = std::make_unique<OneSampleMaterial>(create_lambertian_material(color));
            else
                materials[name] = std::make_unique<OneSampleMaterial>(create_beckmann_glossy_material(color, roughness, ior));
        } else if (b.type == "perspective_camera") {
            Point3  origin{ no_init }, look_at{ no_init };
            Vector3 up{ 0.0f, 1.0f, 0.0f };
            float   fov = 45.0f;
            parse_attrs(b.body, [&](const std::string& k, std::istream& ins) {
                if (k == "origin") ins >> origin;
                else if (k == "look_at") ins >> look_at;
                else if (k == "up") ins >> up;
                else if (k == "fov") ins >> fov;
            });
            camera.reset(new PerspectiveCamera{ origin, look_at, up, Angle{ Degrees{ fov } }, w, h });
        } else if (b.type == "sphere_light") {
            auto transform{ AffineTransformation::identity() };
            RGB  radiance = RGB::white();
            parse_attrs(b.body, [&](const std::string& k, std::istream& ins) {
                if (k == "radiance") ins >> radiance;
                else if (k == "translate") { Vector3 v{ no_init }; ins >> v; transform *= translate(v); }
                else if (k == "rotate") { Vector3 a{ no_init }; Degrees d{ no_init }; ins >> a >> d; transform *= rotate(a, Angle{ d }); }
                else if (k == "scale") { Vector3 v{ no_init }; ins >> v; transform *= scale(v); }
            });
            lights.push_back(std::make_shared<SphereLight>(radiance, transform));
        } else if (b.type == "environment_light") { // FileParser.cpp:325 parse_environment_light
            auto                  transform{ LinearTransformation::identity() };
            RGB                   radiance = RGB::white();
            auto                  max_radiance{ std::numeric_limits<float>::max() };
            std::filesystem::path file{};
            parse_attrs(b.body, [&](const std::string& k, std::istream& ins) {
                if (k == "radiance") ins >> radiance;
                else if (k == "max_radiance") ins >> max_radiance;
                else if (k == "image") ins >> file; // std::filesystem::path >> reads std::quoted
                else if (k == "rotate") { Vector3 a{ no_init }; Degrees d{ no_init }; ins >> a >> d; transform *= rotate(a, Angle{ d }); }
                else if (k == "scale") { Vector3 v{ no_init }; ins >> v; transform *= scale(v); }
                else { std::string r; std::getline(ins, r); }
            });
            if (file.empty()) {
                lights.push_back(std::make_shared<EnvironmentLight>(radiance));
            } else {
                // the reference opens the path relative to the working directory; the harness
                // resolves it against the scene file's directory
                auto img = read(file.is_absolute() ? file : base_dir / file);
                img *= radiance;
                lights.push_back(std::make_shared<ImageBasedEnvironmentLight>(std::move(img), transform, max_radiance));
            }
        }
    }
    for (const auto& b : blocks) { // pass 2: clearcoat materials
        if (b.type != "material_clearcoat") continue;
        std::string               name;
        std::shared_ptr<Material> base;
        float                     ior   = 1.5f;
        RGB                       color = RGB::white();
        parse_attrs(b.body, [&](const std::string& k, std::istream& ins) {
            if (k == "name") { ins >> name; name = trim_quotes(name); }
            else if (k == "base") { std::string m; ins >> m; base = materials.at(trim_quotes(m)); }
            else if (k == "color") ins >> color;
            else if (k == "ior") ins >> ior;
        });
        materials[name] = std::make_unique<ClearcoatMaterial>(create_clearcoat_material(base, ior, color));
    }
    Scene::PrimitiveContainer geometry;
    for (const auto& b : blocks) { // pass 3: geometry in file order
        if (b.type != "mesh" && b.type != "plane" && b.type != "sphere") continue;
        auto                      transform{ AffineTransformation::identity() };
        std::shared_ptr<Material> material;
        std::string               file;
        parse_attrs(b.body, [&](const std::string& k, std::istream& ins) {
            if (k == "material") { std::string m; ins >> m; material = materials.at(trim_quotes(m)); }
            else if (k == "file") { ins >> file; file = trim_quotes(file); }
            else if (k == "translate") { Vector3 v{ no_init }; ins >> v; transform *= translate(v); }
            else if (k == "rotate") { Vector3 a{ no_init }; Degrees d{ no_init }; ins >> a >> d; transform *= rotate(a, Angle{ d }); }
            else if (k == "scale") { Vector3 v{ no_init }; ins >> v; transform *= scale(v); }
        });
        if (b.type == "mesh") {
            const auto fp   = base_dir / file;
            auto       mesh = fp.extension() == ".stl" ? read_stl_mesh(fp, transform) : read_ply_mesh(fp, transform);
            for (std::size_t i = 0; i < mesh->get_num_triangles(); ++i)
                geometry.push_back(std::make_shared<GeometricPrimitive>(std::make_shared<Triangle>(mesh, i), material));
        } else if (b.type == "plane") {
            geometry.push_back(std::make_shared<GeometricPrimitive>(std::make_shared<Plane>(transform), material));
        } else {
            geometry.push_back(std::make_shared<GeometricPrimitive>(std::make_shared<Sphere>(transform), material));
        }
    }
    auto scene                    = std::make_unique<Scene>(geometry.begin(), geometry.end(), lights.begin(), lights.end());
    scene->m_camera               = std::move(camera);
    scene->image_width            = w;
    scene->image_height           = h;
    scene->russian_roulette_depth = rr;
    scene->max_depth              = max_depth;
    return scene;
}

// main.cpp:38-48 create_integrator
std::unique_ptr<Integrator> make_integrator(int type, int w, int h)
{
    switch (static_cast<IntegratorType>(type)) {
    case IntegratorType::Mandelbrot: return std::make_unique<MandelbrotIntegrator>(w, h);
    case IntegratorType::BruteForce: return std::make_unique<BruteForceIntegrator>();
    case IntegratorType::BruteForceIterative: return std::make_unique<BruteForceIntegratorIterative>();
    case IntegratorType::BruteForceIterativeRR: return std::make_unique<BruteForceIntegratorIterativeRR>();
    case IntegratorType::IterativeRRNEE: return std::make_unique<IntegratorIterativeRRNEE>();
    case IntegratorType::DirectLighting: return std::make_unique<DirectLightingIntegrator>();
    case IntegratorType::Whitted: return std::make_unique<WhittedIntegrator>();
    default: return std::make_unique<BruteForceIntegratorIterative>();
    }
}

// main.cpp:86-103 for one tile; the 64 outputs follow TilePixelIterator order (clipped pixels 0)
void render_tile(const Scene& scene, const Integrator& integrator, unsigned spp, int tile_index, MemoryArena& arena,
                 float* out)
{
    const int  tiles_x = (scene.image_width + k_tile_dimension - 1) / k_tile_dimension;
    const Tile full{ Point2i{ (tile_index % tiles_x) * k_tile_dimension, (tile_index / tiles_x) * k_tile_dimension } };
    const Tile tile = intersect(BBox2i{ Point2i{ 0, 0 }, Point2i{ scene.image_width, scene.image_height } }, full);
    int        lane = 0;
    for (auto p : std::views::all(full)) {
        float* o = out + 3 * lane++;
        o[0] = o[1] = o[2] = 0.0f;
        if (!contains(tile, p)) continue;
        auto pixel_sampler      = RSequenceSampler::create_new_sequence(Seed{ static_cast<std::uint32_t>(p.x) << 16u | static_cast<std::uint32_t>(p.y) });
        auto integrator_sampler = IncoherentSampler::create_new_sequence(
            Seed{ (static_cast<std::uint32_t>(p.x) << 16u | static_cast<std::uint32_t>(p.y)) ^ 0xb0ae9d99 });
        RGB acc = RGB::black();
        for (unsigned i = 0; i < spp; ++i) {
            arena.release_all();
            const auto   sample = pixel_sampler.get_next_2D();
            const Point2 pixel_coords{ p.x + sample.x, p.y + sample.y };
            const Ray    ray = scene.m_camera->generate_ray(pixel_coords.x, pixel_coords.y);
            acc += integrator.integrate(ray, scene, arena, integrator_sampler, pixel_coords);
        }
        acc /= spp;
        o[0] = acc.r;
        o[1] = acc.g;
        o[2] = acc.b;
    }
}

} // namespace

extern "C" {

const char* ref_last_error() { return g_error.c_str(); }

// Scene handle: parse + build once (Scene ctor builds the reference BVH), render many times.
void* ref_scene_create(const char* scene_path, int width, int height)
{
    try {
        return build_scene(scene_path, width, height).release();
    } catch (const std::exception& e) {
        g_error = e.what();
        return nullptr;
    }
}

void ref_scene_free(void* scene) { delete static_cast<Scene*>(scene); }

// Render `n_tiles` tiles (ColumnMajorTileScheduler indices) with the reference on `threads`
// threads: out = n_tiles x 64 x 3 floats.  integrator 0 = DirectLighting (main.cpp:387-392).
int ref_render_tiles(void* scene_handle, int integrator, unsigned spp, const int32_t* tile_ids, int64_t n_tiles,
                     int threads, float* out)
{
    try {
        const Scene& scene = *static_cast<Scene*>(scene_handle);
        int          type  = integrator;
        if (type == 0) type = static_cast<int>(IntegratorType::DirectLighting);
        const auto integ = make_integrator(type, scene.image_width, scene.image_height);
        if (threads < 1) threads = 1;
        std::vector<std::thread> pool;
        std::atomic<int64_t>     next{ 0 };
        for (int t = 0; t < threads; ++t) {
            pool.emplace_back([&]() {
                MemoryArena arena;
                for (int64_t i; (i = next++) < n_tiles;) render_tile(scene, *integ, spp, tile_ids[i], arena, out + i * 64 * 3);
            });
        }
        for (auto& t : pool) t.join();
        return 0;
    } catch (const std::exception& e) {
        g_error = e.what();
        return 1;
    }
}

// One-shot convenience: scene file at width x height (<= 0: the file's).  Returns 0 on success.
int ref_render(const char* scene_path, int width, int height, int integrator, unsigned spp, const int32_t* tile_ids,
               int64_t n_tiles, int threads, float* out)
{
    void* sc = ref_scene_create(scene_path, width, height);
    if (!sc) return 1;
    const int rc = ref_render_tiles(sc, integrator, spp, tile_ids, n_tiles, threads, out);
    ref_scene_free(sc);
    return rc;
}

} // extern "C"
