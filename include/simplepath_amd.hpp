// simplepath_amd.hpp -- C++ drop-in for the reference's render path (header-only, C++17).
//
// The reference's main.cpp drives its per-pixel hot path through four names:
//   sp::string_to_integrator_type   Integrators/Integrator.cpp:25
//   sp::Scene / parse_scene_file    base/Scene.h:48, main.cpp:51-65 (sp::parse_file)
//   create_integrator               main.cpp:36-49
//   sp::ColumnMajorTileScheduler    base/TileScheduler.h:59-86
//   render(integrator, threads, spp, scene)   main.cpp:109-141
// This header keeps those names and signatures (namespace sp_amd) over the C-ABI in
// simplepath_hip.h, so main.cpp switches to the MI355X path by changing its namespace for these
// calls.  Every pixel is integrated by HIP kernels on the GPU; no torch, no
// Python.  Errors are thrown as the reference throws them: ParsingException for scene files,
// std::runtime_error("Unknown integrator type") for integrator names, std::runtime_error for
// device failures.
#ifndef SIMPLEPATH_AMD_HPP
#define SIMPLEPATH_AMD_HPP

#include "simplepath_hip.h"

#include <atomic>
#include <cstdint>
#include <memory>
#include <optional>
#include <stdexcept>
#include <string>
#include <utility>
#include <vector>

namespace sp_amd {

// ParsingException (base/FileParser.h:11): messages carry " on line N" like the reference's.
class ParsingException : public std::runtime_error {
public:
    using std::runtime_error::runtime_error;
};

inline void check(int rc)
{
    if (rc == SP_OK) return;
    const std::string msg = sp_last_error();
    if (rc == SP_ERR_PARSE || rc == SP_ERR_IO) throw ParsingException(msg);
    throw std::runtime_error(msg);
}

// IntegratorType (Integrators/Integrator.h:18), same enumerators and order.
enum class IntegratorType : int32_t {
    NotSpecified          = SP_INTEGRATOR_NOT_SPECIFIED,
    Mandelbrot            = SP_INTEGRATOR_MANDELBROT,
    BruteForce            = SP_INTEGRATOR_BRUTE_FORCE,
    BruteForceIterative   = SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE,
    BruteForceIterativeRR = SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE_RR,
    IterativeRRNEE        = SP_INTEGRATOR_ITERATIVE_RRNEE,
    DirectLighting        = SP_INTEGRATOR_DIRECT_LIGHTING,
    Whitted               = SP_INTEGRATOR_WHITTED
};

// string_to_integrator_type (Integrators/Integrator.cpp:25): trims, throws on unknown names.
inline IntegratorType string_to_integrator_type(const std::string& s)
{
    int32_t t = 0;
    if (sp_string_to_integrator(s.c_str(), &t) != SP_OK) throw std::runtime_error("Unknown integrator type");
    return static_cast<IntegratorType>(t);
}

// sp::Scene (base/Scene.h:48) with its public parameters; owns the parsed scene and, once
// uploaded, its HBM copy (BVH, SoA records).  Move-only.
class Scene {
public:
    Scene() = default;
    explicit Scene(sp_scene* s) : m_s(s) { refresh(); }
    Scene(Scene&& o) noexcept { *this = std::move(o); }
    Scene& operator=(Scene&& o) noexcept
    {
        std::swap(m_s, o.m_s);
        image_width            = o.image_width;
        image_height           = o.image_height;
        russian_roulette_depth = o.russian_roulette_depth;
        max_depth              = o.max_depth;
        integrator_type        = o.integrator_type;
        output_file_name       = o.output_file_name;
        return *this;
    }
    Scene(const Scene&)            = delete;
    Scene& operator=(const Scene&) = delete;
    ~Scene() { sp_scene_free(m_s); }

    // Scene::Scene from a scene the host already built (sp_scene_from_desc: arrays copied).
    static Scene from_desc(const sp_scene_desc& d)
    {
        sp_scene* s = nullptr;
        check(sp_scene_from_desc(&d, &s));
        return Scene(s);
    }

    // Override the scene file's image size (the camera is rebuilt as the parser would).
    void set_resolution(int width, int height)
    {
        check(sp_scene_set_resolution(m_s, width, height));
        refresh();
    }
    // HBM residency: bvh_mode 0 = SAH (fast), 1 = the reference's median split (bit-exact order).
    void upload(int device = 0, int bvh_mode = 0) const { check(sp_scene_upload(m_s, device, bvh_mode)); }
    // ... with explicit accelerator options (sp_upload_params, ABI 4)
    void upload(int device, const sp_upload_params& params) const { check(sp_scene_upload_ex(m_s, device, &params)); }
    sp_scene* handle() const noexcept { return m_s; }

    // The reference's public Scene members (base/Scene.h:90-96), as read after loading.  They are
    // snapshots for the host's own use: writing them does not change the render.  The image size
    // is changed with set_resolution; max_depth / russian_roulette_depth / integrator come from
    // the scene file (render with another integrator through Integrator).
    int            image_width            = 0;
    int            image_height           = 0;
    int            russian_roulette_depth = 3;
    int            max_depth              = 10;
    IntegratorType integrator_type        = IntegratorType::NotSpecified;
    std::string    output_file_name;

private:
    void refresh()
    {
        sp_scene_info i{};
        check(sp_scene_get_info(m_s, &i));
        image_width            = i.image_width;
        image_height           = i.image_height;
        russian_roulette_depth = i.russian_roulette_depth;
        max_depth              = i.max_depth;
        integrator_type        = static_cast<IntegratorType>(i.integrator_type);
        output_file_name       = i.output_file_name;
    }
    sp_scene* m_s = nullptr;
};

// parse_scene_file (main.cpp:51-65 -> base/FileParser.cpp:929 sp::parse_file).
inline Scene parse_scene_file(const std::string& file_name)
{
    sp_scene* s = nullptr;
    check(sp_scene_load(file_name.c_str(), &s));
    return Scene(s);
}
// sp::parse_file(std::istream&) on the text of a scene (main.cpp reads "-" from std::cin).
inline Scene parse_scene_text(const std::string& text, const std::string& base_dir = ".")
{
    sp_scene* s = nullptr;
    check(sp_scene_load_string(text.c_str(), base_dir.c_str(), &s));
    return Scene(s);
}

// Integrator (Integrators/Integrator.h:32): which integrate() the device kernels run, plus
// the device pipeline (SP_PIPELINE_*; AUTO picks by work size, all give identical images).
class Integrator {
public:
    explicit Integrator(IntegratorType t, int32_t pipeline = SP_PIPELINE_AUTO) : m_type(t), m_pipeline(pipeline) {}
    IntegratorType type() const noexcept { return m_type; }
    int32_t        pipeline() const noexcept { return m_pipeline; }

private:
    IntegratorType m_type;
    int32_t        m_pipeline;
};

// create_integrator (main.cpp:36-49): NotSpecified falls back to BruteForceIterative as there.
inline std::unique_ptr<Integrator> create_integrator(IntegratorType type, int /*image_width*/, int /*image_height*/,
                                                     int /*russian_roulette_depth*/, int /*max_depth*/)
{
    if (type == IntegratorType::NotSpecified) type = IntegratorType::BruteForceIterative;
    return std::make_unique<Integrator>(type);
}

constexpr int k_tile_dimension = 8; // base/Tile.h:10

// Tile / ScheduledTile (base/Tile.h, base/TileScheduler.h:12): the tile's origin and its
// clipped extent.
struct Tile {
    int x0, y0, x1, y1;
};
struct ScheduledTile {
    Tile tile;
    int  pass;
    int  index; // ColumnMajor tile index: the id sp_render_tiles takes
};

// TileScheduler / ColumnMajorTileScheduler (base/TileScheduler.h:18-86); get_next_tile is
// thread-safe like the reference's (one atomic counter).
class TileScheduler {
public:
    TileScheduler(int width, int height) noexcept : m_w(width), m_h(height) {}
    virtual ~TileScheduler() = default;
    std::optional<ScheduledTile> get_next_tile()
    {
        auto t = get_next_tile_impl();
        if (t) { // intersect(tile, extents)
            t->tile.x1 = t->tile.x1 < m_w ? t->tile.x1 : m_w;
            t->tile.y1 = t->tile.y1 < m_h ? t->tile.y1 : m_h;
        }
        return t;
    }
    int get_num_tiles_x() const noexcept { return (m_w + k_tile_dimension - 1) / k_tile_dimension; }
    int get_num_tiles_y() const noexcept { return (m_h + k_tile_dimension - 1) / k_tile_dimension; }
    int get_num_tiles() const noexcept { return get_num_tiles_x() * get_num_tiles_y(); }

private:
    virtual std::optional<ScheduledTile> get_next_tile_impl() = 0;
    int m_w, m_h;
};

class ColumnMajorTileScheduler : public TileScheduler {
public:
    ColumnMajorTileScheduler(int width, int height, int pass_clamp) noexcept
        : TileScheduler(width, height), m_pass_clamp(pass_clamp)
    {
    }

private:
    std::optional<ScheduledTile> get_next_tile_impl() override
    {
        const int counter   = m_counter++;
        const int num_tiles = get_num_tiles();
        const int pass      = counter / num_tiles;
        if (pass >= m_pass_clamp) return std::nullopt;
        const int index = counter % num_tiles;
        const int x     = (index % get_num_tiles_x()) * k_tile_dimension;
        const int y     = (index / get_num_tiles_x()) * k_tile_dimension;
        return ScheduledTile{ Tile{ x, y, x + k_tile_dimension, y + k_tile_dimension }, pass, index };
    }
    std::atomic<int> m_counter{ 0 };
    int              m_pass_clamp;
};

// sp::Image stand-in: width x height RGB floats, row-major (Image/Image.h).
struct Image {
    int                width = 0, height = 0;
    std::vector<float> rgb;
    float*             operator()(int x, int y) { return &rgb[(static_cast<size_t>(y) * width + x) * 3]; }
};

// The scheduler's tiles (one pass), integrated on the GPU: main.cpp:77-107 render_thread for
// every tile.  The scene is uploaded on first use (SAH BVH unless bvh_mode 1 was uploaded).
inline Image render_image(const Integrator& integrator, unsigned num_pixel_samples, const Scene& scene,
                          sp_render_stats* stats = nullptr)
{
    if (sp_scene_bvh_info(scene.handle(), nullptr, nullptr, nullptr) != SP_OK) scene.upload(0, 0); // not resident yet
    ColumnMajorTileScheduler scheduler{ scene.image_width, scene.image_height, 1 };
    std::vector<int32_t>     ids;
    ids.reserve(static_cast<size_t>(scheduler.get_num_tiles()));
    while (auto t = scheduler.get_next_tile()) ids.push_back(t->index);
    sp_render_params p{};
    p.integrator        = static_cast<int32_t>(integrator.type());
    p.samples_per_pixel = num_pixel_samples;
    p.tile_ids          = ids.data();
    p.num_tiles         = static_cast<int64_t>(ids.size());
    p.flags             = integrator.pipeline();
    std::vector<float> tiles(ids.size() * 64 * 3);
    sp_render_stats    st{};
    check(sp_render_tiles_host(scene.handle(), &p, tiles.data(), &st));
    if (stats) *stats = st;
    Image img;
    img.width  = scene.image_width;
    img.height = scene.image_height;
    img.rgb.assign(static_cast<size_t>(img.width) * img.height * 3, 0.0f);
    check(sp_tiles_to_image(img.width, img.height, ids.data(), p.num_tiles, tiles.data(), img.rgb.data()));
    return img;
}

// render (main.cpp:109-141): integrate every pixel and write scene.output_file_name (PFM,
// Image/Image.cpp:40).  num_threads is accepted for signature compatibility; the GPU does the work.
inline void render(const Integrator& integrator, unsigned /*num_threads*/, unsigned num_pixel_samples, const Scene& scene)
{
    const Image img = render_image(integrator, num_pixel_samples, scene);
    check(sp_write_pfm(scene.output_file_name.c_str(), img.width, img.height, img.rgb.data()));
}

} // namespace sp_amd

#endif // SIMPLEPATH_AMD_HPP
