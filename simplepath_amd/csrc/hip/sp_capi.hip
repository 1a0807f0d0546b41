// sp_capi.hip -- extern "C" boundary (include/simplepath_hip.h) and HBM residency of scenes.
#include "sp_device.hpp"
#include "sp_wave.hpp"
#include "sp_chunk.hpp"
#include "../host/sp_host.hpp"

#include <hip/hip_runtime.h>

#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <stdexcept>
#include <string>
#include <vector>

namespace spd {
hipError_t launch_render(const Scene& sc, const RenderArgs& args, int integ, int variant, int blocks, size_t lds_bytes,
                         hipStream_t stream);
int        render_blocks_per_cu(int integ, int variant, size_t lds_bytes);
size_t     render_static_lds(int integ, int variant);
hipError_t launch_tile_order(float* tile_time, int64_t n_tiles, float factor, int tiles_x, int step, int32_t* order,
                             hipStream_t stream);
bool       has_probe(int integ);
hipError_t launch_probe(const Scene& sc, const RenderArgs& args, int integ, int variant, int blocks, size_t lds_bytes,
                        hipStream_t stream);
hipError_t launch_tail(const Scene& sc, const RenderArgs& args, int variant, int blocks, size_t lds_bytes, hipStream_t stream);
int        tail_blocks_per_cu(int variant, size_t lds_bytes);
} // namespace spd

namespace {
thread_local std::string g_last_error;

int fail(int code, const std::string& msg)
{
    g_last_error = msg;
    return code;
}

#define SP_HIP(call)                                                                                      \
    do {                                                                                                  \
        hipError_t e__ = (call);                                                                          \
        if (e__ != hipSuccess) return fail(SP_ERR_HIP, std::string(#call ": ") + hipGetErrorString(e__)); \
    } while (0)

constexpr int MAX_RECURSION = 32; // sp_path.hpp integrate_bruteforce / integrate_whitted in-register levels

uint32_t code_of(int kind, int index) { return ((uint32_t)kind << spd::CODE_SHIFT) | (uint32_t)index; }

// BBox3 of a primitive (shapes/Triangle.h:228, shapes/Shape.h:290 for transformed shapes)
sph::PrimBounds tri_bounds(const sph::Scene& s, int t)
{
    sph::PrimBounds b;
    for (int i = 0; i < 3; ++i) { b.lo[i] = INFINITY; b.hi[i] = -INFINITY; }
    for (int k = 0; k < 3; ++k) {
        const spm::f3 p   = s.vertices[s.indices[3 * t + k]];
        const float   v[3] = { p.x, p.y, p.z };
        for (int i = 0; i < 3; ++i) {
            b.lo[i] = spm::sse_min(v[i], b.lo[i]); // BBox::extend: min(p, m_min)
            b.hi[i] = spm::sse_max(v[i], b.hi[i]);
        }
    }
    return b;
}

spm::aff from_desc(const sp_affine& d)
{
    spm::aff a;
    a.vx = spm::mk(d.vx[0], d.vx[1], d.vx[2]);
    a.vy = spm::mk(d.vy[0], d.vy[1], d.vy[2]);
    a.vz = spm::mk(d.vz[0], d.vz[1], d.vz[2]);
    a.p  = spm::mk(d.p[0], d.p[1], d.p[2]);
    return a;
}
spm::lin from_desc(const sp_linear& d)
{
    spm::lin a;
    a.vx = spm::mk(d.vx[0], d.vx[1], d.vx[2]);
    a.vy = spm::mk(d.vy[0], d.vy[1], d.vy[2]);
    a.vz = spm::mk(d.vz[0], d.vz[1], d.vz[2]);
    return a;
}

sph::PrimBounds sphere_bounds(const spm::aff& o2w)
{
    sph::PrimBounds b;
    for (int i = 0; i < 3; ++i) { b.lo[i] = INFINITY; b.hi[i] = -INFINITY; }
    // AffineSpace::operator()(BBox3) (math/AffineSpace.h:104): corners p0..p7
    const float lo = -1.0f, hi = 1.0f;
    const float cs[8][3] = { { lo, lo, lo }, { lo, lo, hi }, { lo, hi, lo }, { lo, hi, hi },
                             { hi, lo, lo }, { hi, lo, hi }, { hi, hi, lo }, { hi, hi, hi } };
    for (auto& c : cs) {
        const spm::f3 p    = spm::xfm_point(o2w, spm::mk(c[0], c[1], c[2]));
        const float   v[3] = { p.x, p.y, p.z };
        for (int i = 0; i < 3; ++i) {
            b.lo[i] = spm::sse_min(v[i], b.lo[i]);
            b.hi[i] = spm::sse_max(v[i], b.hi[i]);
        }
    }
    return b;
}

// Accelerator options of an upload (sp_upload_params, ABI 4): explicit fields win; fields left
// automatic take the SP_* environment overrides (test hooks), else the measured defaults.
struct UploadOpts {
    int  bvh_mode   = 0;
    bool stackless  = false; // forced parent-link walk
    int  stack_max  = 96;    // deepest BVH (levels) walked with the LDS stack
    bool wide       = true;  // 8-wide any-hit BVH on SAH scenes
    bool env_guide  = true;  // image-light guide tables
    bool wide_closest = true;  // closest-hit queries on the 8-wide BVH as well
    int  sah_leaf   = 4;
    bool operator==(const UploadOpts& o) const
    {
        return bvh_mode == o.bvh_mode && stackless == o.stackless && stack_max == o.stack_max && wide == o.wide &&
               env_guide == o.env_guide && sah_leaf == o.sah_leaf && wide_closest == o.wide_closest;
    }
};

static int env_int(const char* name, int fallback)
{
    const char* v = std::getenv(name);
    return v ? std::atoi(v) : fallback;
}

int resolve_upload(const sp_upload_params* p, UploadOpts& o)
{
    const sp_upload_params z{};
    if (!p) p = &z;
    if (p->reserved != 0) return fail(SP_ERR_ARG, "sp_upload_params.reserved must be 0");
    if (p->binary_closest != 0 && p->binary_closest != 1) return fail(SP_ERR_ARG, "binary_closest must be 0 or 1");
    if (p->bvh_mode != 0 && p->bvh_mode != 1) return fail(SP_ERR_ARG, "bvh_mode must be 0 (SAH) or 1 (reference)");
    if (p->walk != SP_WALK_AUTO && p->walk != SP_WALK_STACKLESS) return fail(SP_ERR_ARG, "walk must be SP_WALK_AUTO or SP_WALK_STACKLESS");
    if (p->stack_max_levels < 0) return fail(SP_ERR_ARG, "stack_max_levels < 0");
    if (p->sah_leaf < 0 || p->sah_leaf > 4) return fail(SP_ERR_ARG, "sah_leaf must be 0 (automatic) or 1..4");
    o.bvh_mode  = p->bvh_mode;
    o.stackless = p->walk == SP_WALK_STACKLESS || (p->walk == SP_WALK_AUTO && env_int("SP_STACKLESS", 0) != 0);
    o.stack_max = p->stack_max_levels ? p->stack_max_levels : std::max(1, env_int("SP_STACK_MAX", 96));
    o.wide      = !p->no_wide_bvh && env_int("SP_WIDE", 1) != 0;
    o.env_guide = !p->env_replay && env_int("SP_ENV_GUIDE", 1) != 0;
    o.wide_closest = !p->binary_closest && env_int("SP_WIDE_CLOSEST", 1) != 0;
    // SAH leaf size limit (1..4: 8 collapsed leaves of a wide node must fit its 5-bit leaf
    // offsets; the sweep in DESIGN.md §4 found 4 best)
    o.sah_leaf  = p->sah_leaf ? p->sah_leaf : std::max(1, std::min(4, env_int("SP_SAH_LEAF", 4)));
    return SP_OK;
}

// Scene ctor partition (base/Scene.h:29: bounded primitives first, planes after, libstdc++
// std::partition order) and the BVH over the bounded part: the reference's median split
// (bvh_mode 1, shapes/BVHAccelerator.h:173) or SAH.
sph::Bvh geometry_bvh(const sph::Scene& h, const UploadOpts& o, std::vector<int32_t>& prims, size_t& part)
{
    prims.resize(h.prim_kind.size());
    for (size_t i = 0; i < prims.size(); ++i) prims[i] = (int32_t)i;
    part = sph::stl_partition(prims, 0, prims.size(), [&](int32_t p) { return h.prim_kind[p] != SP_PRIM_PLANE; });
    std::vector<sph::PrimBounds> bounds;
    bounds.reserve(part);
    for (size_t i = 0; i < part; ++i) {
        const int32_t p = prims[i];
        if (h.prim_kind[p] == SP_PRIM_TRIANGLE) bounds.push_back(tri_bounds(h, h.prim_index[p]));
        else bounds.push_back(sphere_bounds(from_desc(h.shapes[h.prim_index[p]].object_to_world)));
    }
    return (o.bvh_mode == 1) ? sph::build_bvh_reference(bounds) : sph::build_bvh_sah(bounds, o.sah_leaf);
}

// SAH scenes get the 8-wide quantised BVH for any-hit queries (no_wide_bvh keeps the binary walk)
bool wide_enabled(const UploadOpts& o) { return o.bvh_mode != 1 && o.wide; }

// Traversal-stack budget: a BVH deeper than stack_max levels (default 96) is walked without a
// stack (parent links, sp_path.hpp bvh_next) instead of failing.  96 entries x 4 B x 64 lanes x 4
// waves = 96 KB of LDS, which leaves room for the 16 KB RSQRTSS table and a second block per CU.
bool stackless_for(const UploadOpts& o, int depth) { return o.stackless || depth + 1 > o.stack_max; }

// Scene ctor's light accelerator (base/Scene.h:29): sphere lights first (libstdc++
// std::partition order), the reference BVH over them; the rest are unbounded
sph::Bvh light_bvh(const sph::Scene& h, std::vector<int32_t>& lids, size_t& lpart)
{
    lids.resize(h.lights.size());
    for (size_t i = 0; i < lids.size(); ++i) lids[i] = (int32_t)i;
    lpart = sph::stl_partition(lids, 0, lids.size(), [&](int32_t i) { return h.lights[i].kind == SP_LIGHT_SPHERE; });
    std::vector<sph::PrimBounds> lb;
    for (size_t i = 0; i < lpart; ++i) lb.push_back(sphere_bounds(from_desc(h.lights[lids[i]].object_to_world)));
    return sph::build_bvh_reference(lb);
}

// parent[i] of every node of a binary BVH (the root is its own parent)
std::vector<uint32_t> parent_links(const std::vector<sph::BvhNode>& nodes)
{
    std::vector<uint32_t> par(nodes.size(), 0u);
    for (size_t i = 0; i < nodes.size(); ++i) {
        if (nodes[i].b & sph::BVH_LEAF) continue;
        par[nodes[i].a & sph::BVH_CHILD_MASK] = (uint32_t)i;
        par[nodes[i].b]                       = (uint32_t)i;
    }
    return par;
}

struct DevBuf {
    void*  p     = nullptr;
    size_t bytes = 0;
};
} // namespace

struct sp_scene {
    std::unique_ptr<sph::Scene> host;
    sp_scene_desc               desc{};
    std::vector<sp_env_image>   env_descs; // desc.env_images
    std::vector<sp_material_desc> mat_descs; // desc.materials
    // device residency
    int                  device   = -1;
    int                  bvh_mode = -1;
    UploadOpts           opts{};    // effective accelerator options of the resident upload
    std::vector<DevBuf>  bufs;
    spd::Scene           dev{};
    int                  geom_depth = 0, light_depth = 0;
    size_t               geom_nodes = 0, geom_slots = 0;
    // render scratch
    uint64_t*            mt_state     = nullptr;
    size_t               mt_waves     = 0;
    int32_t*             tile_counter = nullptr;
    unsigned long long*  counters     = nullptr;
    int32_t*             d_tiles      = nullptr;
    size_t               d_tiles_cap  = 0;
    void*                wave_buf     = nullptr; // wavefront pipeline state (sp_wave.hpp WaveArgs)
    size_t               wave_cap     = 0;
    std::vector<hipEvent_t> stage_ev;            // SP_RENDER_STAGE_TIMING
    hipStream_t          aux_stream[spd::WF_MAX_PARTS - 1] = {}; // parts 1.. of the wavefront pipeline
    hipEvent_t           ev_fork = nullptr, ev_join[spd::WF_MAX_PARTS - 1] = {};
    hipEvent_t           ev_shade[spd::WF_MAX_PARTS] = {};
    int                  n_cu         = 0;
    hipEvent_t           ev0 = nullptr, ev1 = nullptr;
    hipEvent_t           ev_render = nullptr; // megakernel, stage timing: before the render launch
    void*                ck_buf     = nullptr; // sample-chunk pipeline: hits, radiance, snapshots
    size_t               ck_cap     = 0;
    int32_t*             ck_ctr     = nullptr;
    void*                deep_buf   = nullptr; // recursive integrators beyond MAX_RECURSION levels
    size_t               deep_cap   = 0;
    float*               d_tile_time = nullptr; // megakernel tile order: probe times, queue order
    int32_t*             d_order     = nullptr;
    size_t               order_cap   = 0;
    unsigned long long*  probe_counters = nullptr;
    void*                tail_buf    = nullptr; // megakernel tail chunks: TailArgs, flags, hits, radiance, store
    size_t               tail_cap    = 0;
    // One scene, many host threads (the reference's render() shares one Scene across N threads,
    // main.cpp:122-130): the render scratch above is per scene, so calls are serialised -- on the
    // host by `mu`, and on the device by making each call's stream wait for the previous call's
    // last operation (ev_done), whichever stream that call used.  A host tile list is staged
    // through a ring of STAGE_RING pinned buffers (h_tiles), each rewritten only once its previous
    // copy has run, so the caller's array may be reused as soon as sp_render_tiles returns.  Each
    // staged copy is queued behind the previous call's render (ev_done), so with one buffer a third
    // back-to-back call waited on the host for the first render; with the ring the host waits only
    // when STAGE_RING calls are queued ahead of the copy it needs.
    static constexpr int STAGE_RING = 4;
    std::mutex           mu;
    hipEvent_t           ev_done  = nullptr; // recorded at the end of every render call
    bool                 done_rec = false;
    int32_t*             h_tiles[STAGE_RING]     = {};  // pinned staging of host tile lists
    size_t               h_tiles_cap[STAGE_RING] = {};
    hipEvent_t           ev_tiles[STAGE_RING]    = {};  // after each buffer's staged copy
    bool                 tiles_rec[STAGE_RING]   = {};
    int                  stage_next = 0;

    void release()
    {
        if (device >= 0) (void)hipSetDevice(device);
        for (auto& b : bufs) (void)hipFree(b.p);
        bufs.clear();
        if (mt_state) (void)hipFree(mt_state);
        if (tile_counter) (void)hipFree(tile_counter);
        if (counters) (void)hipFree(counters);
        if (d_tiles) (void)hipFree(d_tiles);
        if (wave_buf) (void)hipFree(wave_buf);
        wave_buf = nullptr;
        wave_cap = 0;
        for (hipEvent_t e : stage_ev) (void)hipEventDestroy(e);
        stage_ev.clear();
        for (hipStream_t& a : aux_stream) {
            if (a) (void)hipStreamDestroy(a);
            a = nullptr;
        }
        if (ev_fork) (void)hipEventDestroy(ev_fork);
        for (hipEvent_t& e : ev_join) {
            if (e) (void)hipEventDestroy(e);
            e = nullptr;
        }
        for (hipEvent_t& e : ev_shade) {
            if (e) (void)hipEventDestroy(e);
            e = nullptr;
        }
        ev_fork = nullptr;
        if (ev0) (void)hipEventDestroy(ev0);
        if (ev1) (void)hipEventDestroy(ev1);
        if (ev_render) (void)hipEventDestroy(ev_render);
        if (deep_buf) (void)hipFree(deep_buf);
        if (ck_buf) (void)hipFree(ck_buf);
        if (ck_ctr) (void)hipFree(ck_ctr);
        ck_buf = nullptr; ck_ctr = nullptr; ck_cap = 0;
        deep_buf = nullptr; deep_cap = 0;
        if (d_tile_time) (void)hipFree(d_tile_time);
        if (d_order) (void)hipFree(d_order);
        if (probe_counters) (void)hipFree(probe_counters);
        d_tile_time = nullptr; d_order = nullptr; order_cap = 0; probe_counters = nullptr;
        if (tail_buf) (void)hipFree(tail_buf);
        tail_buf = nullptr; tail_cap = 0;
        if (ev_done) (void)hipEventDestroy(ev_done);
        ev_done = nullptr; done_rec = false;
        for (int k = 0; k < STAGE_RING; ++k) {
            if (ev_tiles[k]) (void)hipEventDestroy(ev_tiles[k]);
            if (h_tiles[k]) (void)hipHostFree(h_tiles[k]);
            ev_tiles[k] = nullptr; tiles_rec[k] = false; h_tiles[k] = nullptr; h_tiles_cap[k] = 0;
        }
        stage_next = 0;
        mt_state = nullptr; tile_counter = nullptr; counters = nullptr; d_tiles = nullptr;
        ev0 = ev1 = ev_render = nullptr;
        mt_waves = 0; d_tiles_cap = 0;
        device = -1; bvh_mode = -1;
    }
    ~sp_scene() { release(); }

    template <typename T>
    int upload(const std::vector<T>& v, const T** out)
    {
        *out = nullptr;
        if (v.empty()) return SP_OK;
        DevBuf b;
        b.bytes = v.size() * sizeof(T);
        SP_HIP(hipMalloc(&b.p, b.bytes));
        SP_HIP(hipMemcpy(b.p, v.data(), b.bytes, hipMemcpyHostToDevice));
        bufs.push_back(b);
        *out = static_cast<const T*>(b.p);
        return SP_OK;
    }
};

namespace {
void fill_desc(sp_scene* s)
{
    const sph::Scene& h = *s->host;
    sp_scene_desc&    d = s->desc;
    d                   = sp_scene_desc{};
    d.info.image_width  = h.image_width;
    d.info.image_height = h.image_height;
    d.info.russian_roulette_depth = h.rr_depth;
    d.info.max_depth              = h.max_depth;
    d.info.integrator_type        = h.integrator;
    d.info.num_triangles          = static_cast<int32_t>(h.tri_material.size());
    d.info.num_vertices           = static_cast<int32_t>(h.vertices.size());
    d.info.num_shapes             = static_cast<int32_t>(h.shapes.size());
    d.info.num_lights             = static_cast<int32_t>(h.lights.size());
    d.info.num_materials          = static_cast<int32_t>(h.materials.size());
    std::strncpy(d.info.output_file_name, h.output_file_name.c_str(), sizeof(d.info.output_file_name) - 1);
    auto put = [](float* o, spm::f3 v) { o[0] = v.x; o[1] = v.y; o[2] = v.z; };
    put(d.camera.transform.vx, h.camera.vx);
    put(d.camera.transform.vy, h.camera.vy);
    put(d.camera.transform.vz, h.camera.vz);
    put(d.camera.transform.p, h.camera.p);
    d.camera.film_width  = h.image_width;
    d.camera.film_height = h.image_height;
    static_assert(sizeof(spm::f3) == 12, "f3 packing");
    d.vertices     = h.vertices.empty() ? nullptr : &h.vertices[0].x;
    d.normals      = h.normals.empty() ? nullptr : &h.normals[0].x;
    d.indices      = h.indices.empty() ? nullptr : h.indices.data();
    d.tri_material = h.tri_material.empty() ? nullptr : h.tri_material.data();
    d.shapes       = h.shapes.empty() ? nullptr : h.shapes.data();
    d.prim_kind    = h.prim_kind.empty() ? nullptr : h.prim_kind.data();
    d.prim_index   = h.prim_index.empty() ? nullptr : h.prim_index.data();
    d.num_prims    = static_cast<int64_t>(h.prim_kind.size());
    d.lights       = h.lights.empty() ? nullptr : h.lights.data();
    s->env_descs.clear();
    for (const auto& e : h.env_images) {
        sp_env_image x{};
        x.width        = e.width;
        x.height       = e.height;
        x.pixels       = e.pixels.data();
        x.max_radiance = e.max_radiance;
        put(x.light_to_world.vx, e.light_to_world.vx);
        put(x.light_to_world.vy, e.light_to_world.vy);
        put(x.light_to_world.vz, e.light_to_world.vz);
        put(x.world_to_light.vx, e.world_to_light.vx);
        put(x.world_to_light.vy, e.world_to_light.vy);
        put(x.world_to_light.vz, e.world_to_light.vz);
        s->env_descs.push_back(x);
    }
    s->mat_descs.clear();
    for (const auto& m : h.materials) s->mat_descs.push_back(m.d);
    d.materials      = s->mat_descs.empty() ? nullptr : s->mat_descs.data();
    d.env_images     = s->env_descs.empty() ? nullptr : s->env_descs.data();
    d.num_env_images = static_cast<int32_t>(s->env_descs.size());
}

int wrap_load(std::unique_ptr<sph::Scene> (*fn)(const std::string&, const std::string&), const std::string& a,
              const std::string& b, sp_scene** out)
{
    try {
        auto* s = new sp_scene;
        s->host = fn(a, b);
        fill_desc(s);
        *out = s;
        return SP_OK;
    } catch (const sph::SpError& e) {
        return fail(e.code, e.what());
    } catch (const std::exception& e) {
        return fail(SP_ERR_PARSE, std::string("Unexpected file parsing error: ") + e.what());
    }
}
} // namespace

extern "C" {

const char* sp_version(void) { return "simplepath-amd 0.1 (gfx950)"; }
// content hash of the sources and flags of this build (simplepath_amd/Makefile, ABI 5)
extern const char* const sp_build_id_str;
const char* sp_build_id(void) { return sp_build_id_str; }
const char* sp_last_error(void) { return g_last_error.c_str(); }

int sp_string_to_integrator(const char* name, int32_t* out)
{
    if (!name || !out) return fail(SP_ERR_ARG, "null argument");
    std::string s(name);
    while (!s.empty() && std::isspace(static_cast<unsigned char>(s.back()))) s.pop_back();
    size_t b = 0;
    while (b < s.size() && std::isspace(static_cast<unsigned char>(s[b]))) ++b;
    s = s.substr(b);
    // Integrators/Integrator.cpp:25 string_to_integrator_type
    if (s == "mandelbrot") *out = SP_INTEGRATOR_MANDELBROT;
    else if (s == "brute_force") *out = SP_INTEGRATOR_BRUTE_FORCE;
    else if (s == "brute_force_iterative") *out = SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE;
    else if (s == "brute_force_iterative_rr") *out = SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE_RR;
    else if (s == "iterative_rrnee") *out = SP_INTEGRATOR_ITERATIVE_RRNEE;
    else if (s == "direct_lighting") *out = SP_INTEGRATOR_DIRECT_LIGHTING;
    else if (s == "whitted") *out = SP_INTEGRATOR_WHITTED;
    else return fail(SP_ERR_ARG, "Unknown integrator type");
    return SP_OK;
}

int sp_scene_load(const char* path, sp_scene** out)
{
    if (!path || !out) return fail(SP_ERR_ARG, "null argument");
    return wrap_load([](const std::string& p, const std::string&) { return sph::parse_scene_file(p); }, path, "", out);
}

int sp_scene_load_string(const char* text, const char* base_dir, sp_scene** out)
{
    if (!text || !out) return fail(SP_ERR_ARG, "null argument");
    return wrap_load(&sph::parse_scene, text, base_dir ? base_dir : ".", out);
}

void sp_scene_free(sp_scene* scene) { delete scene; }

int sp_scene_get_info(const sp_scene* scene, sp_scene_info* out)
{
    if (!scene || !out) return fail(SP_ERR_ARG, "null argument");
    *out = scene->desc.info;
    return SP_OK;
}

int sp_scene_get_desc(const sp_scene* scene, sp_scene_desc* out)
{
    if (!scene || !out) return fail(SP_ERR_ARG, "null argument");
    *out = scene->desc; // arrays owned by the scene: valid until sp_scene_free
    return SP_OK;
}

// A host that already built its scene (the reference's main.cpp:368-395 holds an sp::Scene)
// hands it over flattened; nothing is re-parsed.  Every array is copied and checked.
static int scene_from_desc_impl(const sp_scene_desc* d, sp_scene** out)
{
    if (!d || !out) return fail(SP_ERR_ARG, "null argument");
    const sp_scene_info& in = d->info;
    if (in.image_width <= 0 || in.image_height <= 0 || in.image_width > 65535 || in.image_height > 65535)
        return fail(SP_ERR_ARG, "sp_scene_desc: bad image size");
    if (in.num_triangles < 0 || in.num_vertices < 0 || in.num_shapes < 0 || in.num_lights < 0 || in.num_materials < 0 ||
        d->num_prims < 0 || d->num_env_images < 0)
        return fail(SP_ERR_ARG, "sp_scene_desc: negative count");
    auto need = [](const void* p, int64_t n) { return n == 0 || p != nullptr; };
    if (!need(d->vertices, in.num_vertices) || !need(d->normals, in.num_vertices) || !need(d->indices, in.num_triangles) ||
        !need(d->tri_material, in.num_triangles) || !need(d->shapes, in.num_shapes) || !need(d->prim_kind, d->num_prims) ||
        !need(d->prim_index, d->num_prims) || !need(d->lights, in.num_lights) || !need(d->materials, in.num_materials) ||
        !need(d->env_images, d->num_env_images))
        return fail(SP_ERR_ARG, "sp_scene_desc: null array with a nonzero count");
    if (in.integrator_type < SP_INTEGRATOR_NOT_SPECIFIED || in.integrator_type > SP_INTEGRATOR_WHITTED)
        return fail(SP_ERR_ARG, "sp_scene_desc: unknown integrator type");
    auto h             = std::make_unique<sph::Scene>();
    h->image_width     = in.image_width;
    h->image_height    = in.image_height;
    h->rr_depth        = in.russian_roulette_depth;
    h->max_depth       = in.max_depth;
    h->integrator      = in.integrator_type;
    h->output_file_name = std::string(in.output_file_name, strnlen(in.output_file_name, sizeof(in.output_file_name)));
    h->has_camera      = true;
    h->camera_fixed    = true;
    h->camera          = from_desc(d->camera.transform);
    h->vertices.resize((size_t)in.num_vertices);
    h->normals.resize((size_t)in.num_vertices);
    for (int32_t i = 0; i < in.num_vertices; ++i) {
        h->vertices[i] = spm::mk(d->vertices[3 * i], d->vertices[3 * i + 1], d->vertices[3 * i + 2]);
        h->normals[i]  = spm::mk(d->normals[3 * i], d->normals[3 * i + 1], d->normals[3 * i + 2]);
    }
    h->indices.assign(d->indices, d->indices + (size_t)in.num_triangles * 3);
    for (uint32_t v : h->indices)
        if (v >= (uint32_t)in.num_vertices) return fail(SP_ERR_ARG, "sp_scene_desc: vertex index out of range");
    h->tri_material.assign(d->tri_material, d->tri_material + in.num_triangles);
    for (int32_t m : h->tri_material)
        if (m < 0 || m >= in.num_materials) return fail(SP_ERR_ARG, "sp_scene_desc: triangle material out of range");
    h->shapes.assign(d->shapes, d->shapes + in.num_shapes);
    for (const auto& x : h->shapes) {
        if (x.kind != SP_PRIM_SPHERE && x.kind != SP_PRIM_PLANE) return fail(SP_ERR_ARG, "sp_scene_desc: bad shape kind");
        if (x.material < 0 || x.material >= in.num_materials) return fail(SP_ERR_ARG, "sp_scene_desc: shape material out of range");
    }
    h->prim_kind.assign(d->prim_kind, d->prim_kind + d->num_prims);
    h->prim_index.assign(d->prim_index, d->prim_index + d->num_prims);
    for (int64_t i = 0; i < d->num_prims; ++i) {
        const int k = h->prim_kind[i], x = h->prim_index[i];
        const int n = (k == SP_PRIM_TRIANGLE) ? in.num_triangles : in.num_shapes;
        if ((k != SP_PRIM_TRIANGLE && k != SP_PRIM_SPHERE && k != SP_PRIM_PLANE) || x < 0 || x >= n ||
            (k != SP_PRIM_TRIANGLE && h->shapes[x].kind != k))
            return fail(SP_ERR_ARG, "sp_scene_desc: bad primitive reference");
    }
    for (int32_t i = 0; i < in.num_materials; ++i) {
        const sp_material_desc& m = d->materials[i];
        if (m.kind < SP_MAT_LAMBERTIAN || m.kind > SP_MAT_CLEARCOAT ||
            (m.kind == SP_MAT_CLEARCOAT && (m.base < 0 || m.base >= in.num_materials)))
            return fail(SP_ERR_ARG, "sp_scene_desc: bad material");
        h->materials.push_back(sph::Material{ m });
        h->material_names.push_back(std::string());
    }
    for (int32_t i = 0; i < d->num_env_images; ++i) {
        const sp_env_image& e = d->env_images[i];
        if (e.width <= 0 || e.height <= 0 || !e.pixels) return fail(SP_ERR_ARG, "sp_scene_desc: bad environment image");
        sph::EnvImage x;
        x.width        = e.width;
        x.height       = e.height;
        x.pixels.assign(e.pixels, e.pixels + (size_t)e.width * e.height * 3);
        x.max_radiance = e.max_radiance;
        x.light_to_world = from_desc(e.light_to_world);
        x.world_to_light = from_desc(e.world_to_light);
        h->env_images.push_back(std::move(x));
    }
    h->lights.assign(d->lights, d->lights + in.num_lights);
    for (const auto& l : h->lights) {
        if (l.kind < SP_LIGHT_SPHERE || l.kind > SP_LIGHT_IMAGE_ENVIRONMENT) return fail(SP_ERR_ARG, "sp_scene_desc: bad light kind");
        if (l.kind == SP_LIGHT_IMAGE_ENVIRONMENT && (l.image < 0 || l.image >= d->num_env_images))
            return fail(SP_ERR_ARG, "sp_scene_desc: light image out of range");
    }
    auto* s = new sp_scene;
    s->host = std::move(h);
    fill_desc(s);
    *out = s;
    return SP_OK;
}

int sp_scene_from_desc(const sp_scene_desc* d, sp_scene** out)
{
    try {
        return scene_from_desc_impl(d, out);
    } catch (const std::exception& e) {
        return fail(SP_ERR_ARG, std::string("sp_scene_from_desc: ") + e.what());
    }
}

int sp_scene_set_resolution(sp_scene* scene, int32_t width, int32_t height)
{
    if (!scene || width <= 0 || height <= 0 || width > 65535 || height > 65535) return fail(SP_ERR_ARG, "bad resolution");
    if (scene->host->camera_fixed && (width != scene->host->image_width || height != scene->host->image_height))
        return fail(SP_ERR_STATE, "scene built from a descriptor: its camera transform fixes the image size");
    scene->host->image_width  = width;
    scene->host->image_height = height;
    scene->host->rebuild_camera();
    fill_desc(scene);
    if (scene->device >= 0) {
        scene->dev.width  = width;
        scene->dev.height = height;
        scene->dev.camera = scene->host->camera;
    }
    return SP_OK;
}

int sp_tile_count(int32_t width, int32_t height, int64_t* out)
{
    if (!out || width < 0 || height < 0) return fail(SP_ERR_ARG, "bad argument");
    *out = (int64_t)((width + 7) / 8) * ((height + 7) / 8);
    return SP_OK;
}

int sp_tile_origin(int32_t width, int32_t height, int64_t tile, int32_t* x0, int32_t* y0)
{
    int64_t n;
    sp_tile_count(width, height, &n);
    if (tile < 0 || tile >= n || !x0 || !y0) return fail(SP_ERR_ARG, "tile out of range");
    const int32_t w = (width + 7) / 8;
    *x0             = (int32_t)(tile % w) * 8;
    *y0             = (int32_t)(tile / w) * 8;
    return SP_OK;
}

int sp_device_count(int32_t* out)
{
    if (!out) return fail(SP_ERR_ARG, "null argument");
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
    *out = n;
    return SP_OK;
}

int sp_rsqrt_table_info(int32_t* mantissa_bits, int32_t* verified)
{
    const auto& c = sph::rsqrt_capture();
    if (mantissa_bits) *mantissa_bits = c.bits;
    if (verified) *verified = c.verified ? 1 : 0;
    return SP_OK;
}

int sp_rsqrt_table_get(uint32_t* entries, int64_t capacity, int32_t* bits, uint32_t* zero_result,
                       uint32_t* denorm_result)
{
    const auto& c = sph::rsqrt_active();
    if (c.entries.empty()) return fail(SP_ERR_UNSUPPORTED, "RSQRTSS table capture failed");
    if (bits) *bits = c.bits;
    if (zero_result) *zero_result = c.zero_result;
    if (denorm_result) *denorm_result = c.denorm_result;
    if (entries) {
        if (capacity < (int64_t)c.entries.size()) return fail(SP_ERR_ARG, "RSQRTSS table: capacity too small");
        std::memcpy(entries, c.entries.data(), c.entries.size() * sizeof(uint32_t));
    }
    return SP_OK;
}

int sp_rsqrt_table_set(const uint32_t* entries, int32_t bits, uint32_t zero_result, uint32_t denorm_result)
{
    try {
        sph::rsqrt_set_override(entries, bits, zero_result, denorm_result);
        return SP_OK;
    } catch (const sph::SpError& e) {
        return fail(e.code, e.what());
    }
}

float sp_host_rsqrt_emulated(float x)
{
    const auto&     c = sph::rsqrt_capture();
    spm::RsqrtTable t{ c.entries.data(), c.bits, c.zero_result, c.denorm_result };
    return spm::rsqrtss_emulated(x, t);
}

// Words of LDS traversal stack per lane.  The binary walks push at most one deferred child per
// level; the wide walks one child group per level, and the closest-hit form keeps each group's
// entry distance in the upper half.  Once closest hits walk the wide BVH (SAH scenes), no query
// walks the binary geometry BVH, so its depth no longer sizes the stack -- only the wide and the
// light BVH's do (lucy 30 -> 22 words: a fourth 4-wave block fits a CU's LDS).
static int stack_entries(int depth, int wide_depth, int light_depth, bool wide_closest)
{
    if (wide_closest) return std::max(2 * (wide_depth + 1), light_depth + 1);
    return std::max(depth, std::max(wide_depth, light_depth)) + 1;
}

static int scene_upload_impl(sp_scene* s, int32_t device, const sp_upload_params* up_params)
{
    if (!s) return fail(SP_ERR_ARG, "null scene");
    UploadOpts opts;
    if (int rc0 = resolve_upload(up_params, opts)) return rc0;
    const int bvh_mode = opts.bvh_mode;
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev == 0) return fail(SP_ERR_HIP, "no HIP device");
    if (device < 0 || device >= ndev) return fail(SP_ERR_ARG, "device out of range");
    if (s->device == device && s->opts == opts) return SP_OK;
    s->release();
    SP_HIP(hipSetDevice(device));
    s->device   = device;
    s->bvh_mode = bvh_mode;
    s->opts     = opts;
    const sph::Scene& h = *s->host;
    spd::Scene&       d = s->dev;
    d                   = spd::Scene{};

    const auto& rc = sph::rsqrt_active();
    if (rc.entries.empty()) return fail(SP_ERR_UNSUPPORTED, "RSQRTSS table capture failed");
    if (!rc.verified) return fail(SP_ERR_UNSUPPORTED, "RSQRTSS table could not be verified on this host CPU");

    // ---- materials (nested clearcoat is not produced by the scenes on this path)
    std::vector<spd::Material> mats;
    for (auto& m : h.materials) {
        spd::Material x{};
        x.kind           = m.d.kind;
        x.base           = m.d.base;
        x.lambert_albedo = spm::mkc(m.d.lambert_albedo[0], m.d.lambert_albedo[1], m.d.lambert_albedo[2]);
        x.microfacet_r   = spm::mkc(m.d.microfacet_r[0], m.d.microfacet_r[1], m.d.microfacet_r[2]);
        x.alpha_x        = m.d.alpha_x;
        x.alpha_y        = m.d.alpha_y;
        x.microfacet_ior = m.d.microfacet_ior;
        x.sample_visible_area = m.d.sample_visible_area;
        x.coat_ior       = m.d.coat_ior;
        x.coat_color     = spm::mkc(m.d.coat_color[0], m.d.coat_color[1], m.d.coat_color[2]);
        if (x.kind == SP_MAT_CLEARCOAT && h.materials[x.base].d.kind == SP_MAT_CLEARCOAT)
            return fail(SP_ERR_UNSUPPORTED, "clearcoat over clearcoat");
        mats.push_back(x);
    }

    // ---- geometry: Scene ctor partition (base/Scene.h:29) then BVH over the bounded part
    std::vector<int32_t> prims;
    size_t               part = 0;
    const sph::Bvh       bvh  = geometry_bvh(h, opts, prims, part);
    std::vector<spd::Shape> shapes;
    for (auto& sh : h.shapes) {
        spd::Shape x{};
        x.o2w      = from_desc(sh.object_to_world);
        x.w2o      = from_desc(sh.world_to_object);
        x.nrm      = from_desc(sh.normal_to_world);
        x.material = sh.material;
        x.kind     = sh.kind;
        shapes.push_back(x);
    }
    std::vector<int32_t> unbounded;
    for (size_t i = part; i < prims.size(); ++i) unbounded.push_back(h.prim_index[prims[i]]);
    std::vector<float4>   slot_tri(bvh.prim_order.size() * 3);
    std::vector<uint32_t> slot_code(bvh.prim_order.size());
    for (size_t sl = 0; sl < bvh.prim_order.size(); ++sl) {
        const int32_t p    = prims[bvh.prim_order[sl]];
        const int     kind = h.prim_kind[p];
        const int     idx  = h.prim_index[p];
        slot_code[sl]      = code_of(kind, idx);
        if (kind == SP_PRIM_TRIANGLE) {
            for (int k = 0; k < 3; ++k) {
                const spm::f3 v  = h.vertices[h.indices[3 * idx + k]];
                slot_tri[3 * sl + k] = make_float4(v.x, v.y, v.z, 0.0f);
            }
        }
        // the primitive code rides in p0.w so a triangle test is three 16-byte fetches
        uint32_t code = slot_code[sl];
        std::memcpy(&slot_tri[3 * sl].w, &code, 4);
    }
    std::vector<spd::Node> nodes(bvh.nodes.size());
    static_assert(sizeof(spd::Node) == sizeof(sph::BvhNode), "node layout");
    std::memcpy(nodes.data(), bvh.nodes.data(), nodes.size() * sizeof(spd::Node));
    // ---- lights: Scene::m_lights order + accelerator (partition by boundedness)
    std::vector<spd::Light> lights;
    for (auto& l : h.lights) {
        spd::Light x{};
        x.kind     = l.kind;
        x.image    = l.kind == SP_LIGHT_IMAGE_ENVIRONMENT ? l.image : -1;
        x.radiance = spm::mkc(l.radiance[0], l.radiance[1], l.radiance[2]);
        x.o2w      = from_desc(l.object_to_world);
        x.w2o      = from_desc(l.world_to_object);
        x.nrm      = from_desc(l.normal_to_world);
        lights.push_back(x);
    }
    std::vector<int32_t> lids;
    size_t               lpart = 0;
    const sph::Bvh       lbvh  = light_bvh(h, lids, lpart);
    std::vector<int32_t> unbounded_lights(lids.begin() + (long)lpart, lids.end());
    std::vector<uint32_t> light_slot(lbvh.prim_order.size());
    for (size_t sl = 0; sl < light_slot.size(); ++sl) light_slot[sl] = (uint32_t)lids[lbvh.prim_order[sl]];
    std::vector<spd::Node> lnodes(lbvh.nodes.size());
    std::memcpy(lnodes.data(), lbvh.nodes.data(), lnodes.size() * sizeof(spd::Node));

    // SAH: 8-wide quantised BVH for any-hit queries (SP_WIDE=0 keeps the binary walk); a
    // stackless scene walks the binary BVH only
    const bool          stackless = stackless_for(opts, std::max(bvh.max_depth, lbvh.max_depth));
    sph::WideBvh        wide;
    std::vector<float4> wslot_tri;
    if (wide_enabled(opts) && !nodes.empty() && !stackless) {
        wide = sph::build_wide(bvh);
        wslot_tri.resize(wide.slot_of.size() * 3);
        for (size_t i = 0; i < wide.slot_of.size(); ++i)
            for (int k = 0; k < 3; ++k) wslot_tri[3 * i + k] = slot_tri[3 * (size_t)wide.slot_of[i] + k];
    }

    // ---- upload
    int rc2 = SP_OK;
    auto up = [&](auto& vec, auto** ptr) { if (rc2 == SP_OK) rc2 = s->upload(vec, ptr); };
    d.camera    = h.camera;
    d.width     = h.image_width;
    d.height    = h.image_height;
    d.max_depth = h.max_depth;
    d.rr_depth  = h.rr_depth;
    float a1[1], a2[2];
    sph::rsequence_alphas(a1, a2);
    d.alpha2_0 = a2[0];
    d.alpha2_1 = a2[1];
    d.n_unbounded = (int)unbounded.size();
    up(unbounded, &d.unbounded);
    d.n_nodes = (int)nodes.size();
    up(nodes, &d.nodes);
    d.wnodes    = nullptr;
    d.wslot_tri = nullptr;
    if (!wide.words.empty()) {
        std::vector<uint4> wn(wide.words.size() / 4);
        std::memcpy(wn.data(), wide.words.data(), wide.words.size() * 4);
        up(wn, &d.wnodes);
        up(wslot_tri, &d.wslot_tri);
    }
    up(slot_tri, &d.slot_tri);
    up(slot_code, &d.slot_code);
    std::vector<float> nrm(h.normals.size() * 3);
    for (size_t i = 0; i < h.normals.size(); ++i) { nrm[3 * i] = h.normals[i].x; nrm[3 * i + 1] = h.normals[i].y; nrm[3 * i + 2] = h.normals[i].z; }
    up(nrm, &d.normals);
    up(h.indices, &d.indices);
    up(h.tri_material, &d.tri_material);
    up(shapes, &d.shapes);
    d.n_lights = (int)lights.size();
    up(lights, &d.lights);
    d.n_unbounded_lights = (int)unbounded_lights.size();
    up(unbounded_lights, &d.unbounded_lights);
    d.n_light_nodes = (int)lnodes.size();
    up(lnodes, &d.light_nodes);
    up(light_slot, &d.light_slot);
    // image environment lights: the constructor's tables (sp_envmap.cpp), then the EnvMap records
    std::vector<spd::EnvMap> envs;
    for (const auto& e : h.env_images) {
        const sph::EnvMap m = sph::build_env_map(e);
        spd::EnvMap       x{};
        x.l2w = e.light_to_world;
        x.w2l = e.world_to_light;
        x.w = m.w; x.h = m.h; x.nu = m.nu; x.nv = m.nv;
        std::vector<float4> rad((size_t)m.w * m.h);
        for (size_t i = 0; i < rad.size(); ++i) rad[i] = make_float4(m.radiance[3 * i], m.radiance[3 * i + 1], m.radiance[3 * i + 2], 0.0f);
        up(rad, &x.radiance);
        up(m.cond_func, &x.cond_func);
        up(m.cond_cdf, &x.cond_cdf);
        up(m.cond_int, &x.cond_int);
        up(m.marg_func, &x.marg_func);
        up(m.marg_cdf, &x.marg_cdf);
        x.marg_int   = m.marg_int;
        x.cond_guide = nullptr;
        x.marg_guide = nullptr;
        x.cond_bits  = m.cond_bits;
        x.marg_bits  = m.marg_bits;
        if (m.guided && opts.env_guide) { // else the exact upper_bound replay (identical results)
            up(m.cond_guide, &x.cond_guide);
            up(m.marg_guide, &x.marg_guide);
        }
        envs.push_back(x);
    }
    d.envs = nullptr;
    up(envs, &d.envs);
    up(mats, &d.materials);
    // RSQRTSS table as 16-bit device entries when every entry has the same sign and exponent and
    // at least 7 trailing zero mantissa bits (Intel and AMD hosts alike: exponent 126, 12
    // significant bits): half the LDS each shading block copies it into (sp_math.h).
    int      rs_shift = 23;
    uint32_t rs_hi    = rc.entries[0] & 0xff800000u;
    for (uint32_t e : rc.entries) {
        if ((e & 0xff800000u) != rs_hi) {
            rs_shift = 0;
            break;
        }
        while (rs_shift > 0 && (e & ((1u << rs_shift) - 1u))) --rs_shift;
    }
    if (const char* v = std::getenv("SP_RSQRT_PACK")) // 0: 32-bit entries (comparison)
        if (std::atoi(v) == 0) rs_shift = 0;
    if (rs_shift < 7) rs_shift = 0;
    {
        const uint32_t hdr[spd::RSQ_HDR] = { (uint32_t)rc.bits, rc.zero_result, rc.denorm_result, (uint32_t)rs_shift,
                                             rs_shift ? rs_hi : 0u, 0u, 0u, 0u };
        std::vector<uint32_t> words(hdr, hdr + spd::RSQ_HDR);
        if (rs_shift) {
            std::vector<uint16_t> packed(rc.entries.size());
            for (size_t i = 0; i < packed.size(); ++i) packed[i] = (uint16_t)((rc.entries[i] & 0x7fffffu) >> rs_shift);
            words.resize(spd::RSQ_HDR + (packed.size() + 1) / 2, 0u);
            std::memcpy(words.data() + spd::RSQ_HDR, packed.data(), packed.size() * sizeof(uint16_t));
        } else {
            words.insert(words.end(), rc.entries.begin(), rc.entries.end());
        }
        up(words, &d.rsqrt_entries);
    }
    if (rc2 != SP_OK) return rc2;
    d.rsqrt_shift  = rs_shift;
    d.rsqrt_hi     = rs_shift ? rs_hi : 0u;
    d.rsqrt_bits   = rc.bits;
    d.rsqrt_zero   = rc.zero_result;
    d.rsqrt_denorm = rc.denorm_result;
    s->geom_depth  = bvh.max_depth;
    s->light_depth = lbvh.max_depth;
    s->geom_nodes  = nodes.size();
    s->geom_slots  = slot_code.size();
    // SAH scenes walk the 8-wide BVH for every query: any-hit since round 1 (shadow stage 0.82 ->
    // 0.53 ms), closest hit since round 3 with octant-ordered slots, near-first entry and group
    // distances (bunny 3110 -> 3200, lucy 2175 -> 2280 Mrays/s).  Its stack keeps a
    // distance per entry in the upper half.
    d.ordered     = bvh_mode == 1 ? 0 : 1; // reference order is part of the bit-exact contract
    d.wide_closest = (opts.wide_closest && !wide.words.empty()) ? 1 : 0;
    d.stack_depth  = stack_entries(bvh.max_depth, wide.depth, lbvh.max_depth, d.wide_closest != 0);
    d.stackless   = stackless ? 1 : 0;
    d.merge_queries = 1; // per render: SP_RENDER_PER_LANE_QUERIES clears it
    d.parents       = nullptr;
    d.light_parents = nullptr;
    if (d.stackless) { // deeper than the LDS budget: parent links instead of a stack
        std::vector<uint32_t> par  = parent_links(bvh.nodes);
        std::vector<uint32_t> lpar = parent_links(lbvh.nodes);
        up(par, &d.parents);
        up(lpar, &d.light_parents);
        if (rc2 != SP_OK) return rc2;
        d.stack_depth = 0;
    }
    d.stack_words     = d.stack_depth;
    d.any_stack_words = d.stackless ? 0 : std::max(wide.words.empty() ? bvh.max_depth : wide.depth, lbvh.max_depth) + 1;
    SP_HIP(hipMalloc(&s->tile_counter, sizeof(int32_t)));
    SP_HIP(hipMalloc(&s->counters, 8 * sizeof(unsigned long long)));
    SP_HIP(hipEventCreate(&s->ev0));
    SP_HIP(hipEventCreate(&s->ev1));
    SP_HIP(hipEventCreateWithFlags(&s->ev_done, hipEventDisableTiming));
    for (hipEvent_t& e : s->ev_tiles) SP_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
    return SP_OK;
}

// No C++ exception crosses the C ABI: host-side failures (allocation, BVH encoding limits)
// come back as error codes with sp_last_error() set.
int sp_scene_upload_ex(sp_scene* s, int32_t device, const sp_upload_params* params)
{
    if (!s) return fail(SP_ERR_ARG, "null scene");
    std::lock_guard<std::mutex> lock(s->mu);
    try {
        return scene_upload_impl(s, device, params);
    } catch (const sph::SpError& e) {
        return fail(e.code, e.what());
    } catch (const std::exception& e) {
        return fail(SP_ERR_UNSUPPORTED, std::string("scene upload failed: ") + e.what());
    }
}

int sp_scene_upload(sp_scene* s, int32_t device, int32_t bvh_mode)
{
    sp_upload_params p{};
    p.bvh_mode = bvh_mode;
    return sp_scene_upload_ex(s, device, &p);
}

static int render_tiles_impl(sp_scene* s, const sp_render_params* p, float* d_out, sp_render_stats* stats);
int sp_render_tiles(sp_scene* s, const sp_render_params* p, float* d_out, sp_render_stats* stats)
{
    if (!s) return fail(SP_ERR_ARG, "null argument");
    std::lock_guard<std::mutex> lock(s->mu); // calls on one scene run one at a time (sp_scene::mu)
    try {
        return render_tiles_impl(s, p, d_out, stats);
    } catch (const sph::SpError& e) {
        return fail(e.code, e.what());
    } catch (const std::exception& e) {
        return fail(SP_ERR_HIP, std::string("render failed: ") + e.what());
    }
}

// Megakernel tail chunks (render_tiles_impl): the fraction of the tiles cut into sample chunks at
// the end of the queue, and chunks per tile.
#ifndef SP_TAIL_FRAC
#define SP_TAIL_FRAC 0.12f
#endif
#ifndef SP_TAIL_CHUNKS
#define SP_TAIL_CHUNKS 64
#endif
// The sample-chunk pipeline's fused form (render_tiles_impl): on, and the preps placed ahead of the
// first chunks = persistent waves / SP_CK_FRONT_DIV
#ifndef SP_CK_FUSED
#define SP_CK_FUSED 1
#endif
#ifndef SP_CK_CAMFOLD
#define SP_CK_CAMFOLD 1
#endif
#ifndef SP_CK_CAM_BLOCK
#define SP_CK_CAM_BLOCK 32
#endif
#ifndef SP_CK_FRONT_DIV
#define SP_CK_FRONT_DIV 8
#endif

// Sample-chunk buffer plan (sp_chunk.hip): the same sizes decide AUTO and are allocated.
struct ChunkPlan {
    int64_t  chunks = 1;    // chunks per pixel
    uint32_t len = 1;       // samples per chunk (the last may be short)
    uint32_t gens = 0;      // generator-store generations per pixel
    bool     known_draws = true;
    size_t   b_hits = 0, b_L = 0, b_snap = 0, b_ctl = 0, b_draws = 0, total = 0;
};
static ChunkPlan chunk_plan(const sp_scene* s, int64_t n_tiles, uint32_t spp, int64_t chunks_req)
{
    ChunkPlan c;
    // chunks per pixel: the smallest power of two (<= 32) giving ~120K (tile, chunk) items (the
    // best of the bunny 2/4/8-way shard sweep) unless the caller asks for a count
    c.chunks = 1;
    while (c.chunks < 32 && n_tiles * c.chunks < 120000) c.chunks *= 2;
    if (chunks_req > 0) c.chunks = chunks_req;
    c.chunks = std::min<int64_t>(c.chunks, spp);
    c.len    = (uint32_t)((spp + c.chunks - 1) / c.chunks);
    c.chunks = (spp + c.len - 1) / c.len;
    // a DirectLighting sample draws at most 34 words per light (Light::sample 2 + glossy rho 32);
    // +2 generations for the first twist and the one rng_prepare may twist ahead
    const uint64_t max_draws = (uint64_t)spp * (uint64_t)std::max(1, s->dev.n_lights) * 34;
    c.gens = (uint32_t)((max_draws + spm::MT_N - 1) / spm::MT_N + 2);
    // per-sample draw counts from the camera pass unless an image light makes them depend on the
    // drawn numbers (then ck_count replays Light::sample); SP_CHUNK_REPLAY=1 forces the replay (test)
    c.known_draws = s->dev.n_lights <= 1000;
    for (const auto& l : s->host->lights)
        if (l.kind == SP_LIGHT_IMAGE_ENVIRONMENT) c.known_draws = false;
    if (const char* v = std::getenv("SP_CHUNK_REPLAY")) c.known_draws = c.known_draws && std::atoi(v) == 0;
    const size_t n_px = (size_t)n_tiles * 64;
    c.b_hits  = n_px * spp * 16;
    c.b_L     = n_px * spp * 12;
    c.b_snap  = (size_t)n_tiles * c.gens * spd::MT_GEN_WORDS * 8;
    c.b_ctl   = (size_t)c.chunks * n_px * 4;
    c.b_draws = c.known_draws ? n_px * spp * 2 : 0;
    c.total   = c.b_hits + c.b_L + c.b_snap + c.b_ctl + c.b_draws + 4 * 256;
    return c;
}

// Queue neighbours of the tile-order kernel's cost estimate (sp_mega.hip tile_est): > 0 the queue
// offset of the tile below, -1 the +-1 queue neighbours only, 0 none.  The tile ids are row-major
// (base/TileScheduler.h:75-77: x = index % tiles_x), so for a whole frame (k = 1) the +-1 queue
// neighbours are the tiles left and right.  For a host list with a constant stride k > 1 (a rank's
// interleaved shard) they are the tiles k columns to the left and right -- the same row, not
// adjacent -- and the tile below is tiles_x / k entries on when k divides tiles_x; otherwise
// (-1) the rows of consecutive entries shift and only the +-1 entries are used.  SP_TILE_STRIDE_ROW
// 0 drops the +-1 entries for k > 1 (the column blend alone, or the probe time alone when k does
// not divide tiles_x).  Row blend kept for k > 1 by an A/B on elf's 8-way shard.
#ifndef SP_TILE_STRIDE_ROW
#define SP_TILE_STRIDE_ROW 1
#endif
static int order_neighbours(const sp_render_params* p, bool listed, int64_t n_tiles, int32_t tiles_x)
{
    if (!listed) return tiles_x;
    if (!p->tile_ids || n_tiles < 2) return 0;
    const int64_t k = (int64_t)p->tile_ids[1] - p->tile_ids[0];
    if (k <= 0) return 0;
    for (int64_t i = 2; i < n_tiles; ++i)
        if ((int64_t)p->tile_ids[i] - p->tile_ids[i - 1] != k) return 0;
    if (k > 1 && !SP_TILE_STRIDE_ROW) return (tiles_x % k == 0) ? -(int)(tiles_x / k) - 1 : 0;
    return (tiles_x % k == 0) ? (int)(tiles_x / k) : -1;
}

static int render_tiles_impl(sp_scene* s, const sp_render_params* p, float* d_out, sp_render_stats* stats)
{
    if (!s || !p || !d_out) return fail(SP_ERR_ARG, "null argument");
    if (s->device < 0) return fail(SP_ERR_STATE, "sp_scene_upload must be called before sp_render_tiles");
    if (p->samples_per_pixel == 0) return fail(SP_ERR_ARG, "samples_per_pixel must be > 0");
    if (p->reserved != 0) return fail(SP_ERR_ARG, "sp_render_params.reserved must be 0");
    if (!(p->tail_fraction <= 1.0f)) return fail(SP_ERR_ARG, "tail_fraction must be at most 1 (and not NaN)");
    if (p->tile_ids && p->d_tile_ids) return fail(SP_ERR_ARG, "give tile_ids (host) or d_tile_ids (device), not both");
    if (p->chunks_per_pixel < 0) return fail(SP_ERR_ARG, "chunks_per_pixel < 0");
    if (!(p->chunk_max_gb >= 0.0f)) return fail(SP_ERR_ARG, "chunk_max_gb < 0");
    if (p->tile_order_factor != p->tile_order_factor) return fail(SP_ERR_ARG, "tile_order_factor is NaN");
    if ((p->flags & ~(3 | SP_RENDER_STAGE_TIMING | SP_RENDER_PER_LANE_QUERIES)) != 0) return fail(SP_ERR_ARG, "unknown flags");
    SP_HIP(hipSetDevice(s->device));
    int32_t integ = p->integrator;
    if (integ == SP_INTEGRATOR_NOT_SPECIFIED) integ = s->host->integrator;
    if (integ == SP_INTEGRATOR_NOT_SPECIFIED) integ = SP_INTEGRATOR_DIRECT_LIGHTING; // main.cpp:390
    if (integ < SP_INTEGRATOR_MANDELBROT || integ > SP_INTEGRATOR_WHITTED) return fail(SP_ERR_ARG, "Unknown integrator type");
    // megakernel occupancy request: DirectLighting 1..4 waves per SIMD, IterativeRRNEE 2..4;
    // the other integrators have one variant each (0 = automatic)
    const int waves_req = p->waves_per_simd;
    if (waves_req != 0) {
        const bool ok = integ == SP_INTEGRATOR_DIRECT_LIGHTING ? (waves_req >= 1 && waves_req <= 4)
                        : integ == SP_INTEGRATOR_ITERATIVE_RRNEE ? (waves_req >= 2 && waves_req <= 4)
                                                                  : false;
        if (!ok) return fail(SP_ERR_ARG, "waves_per_simd: DirectLighting 1-4, IterativeRRNEE 2-4, else 0");
    }
    int64_t total;
    sp_tile_count(s->dev.width, s->dev.height, &total);
    const bool    listed  = p->tile_ids || p->d_tile_ids;
    const int64_t n_tiles = listed ? p->num_tiles : total;
    if (n_tiles < 0) return fail(SP_ERR_ARG, "num_tiles < 0");
    if (p->tile_ids)
        for (int64_t i = 0; i < n_tiles; ++i)
            if (p->tile_ids[i] < 0 || p->tile_ids[i] >= total) return fail(SP_ERR_ARG, "tile id out of range");
    hipStream_t stream = static_cast<hipStream_t>(p->stream);
    if (stats) *stats = sp_render_stats{};
    if (n_tiles == 0) return SP_OK;
    // the previous call on this scene may have used another stream: its work on the shared
    // scratch comes first (sp_scene::mu)
    if (s->done_rec) SP_HIP(hipStreamWaitEvent(stream, s->ev_done, 0));
    const int32_t* d_ids = p->d_tile_ids; // device tile list (nullptr: slot = tile)
    if (p->tile_ids) {
        if ((size_t)n_tiles > s->d_tiles_cap) {
            if (s->d_tiles) (void)hipFree(s->d_tiles);
            s->d_tiles = nullptr;
            SP_HIP(hipMalloc(&s->d_tiles, (size_t)n_tiles * sizeof(int32_t)));
            s->d_tiles_cap = (size_t)n_tiles;
        }
        // staged through the next pinned buffer of the ring, so the caller's array is free once this
        // returns; the host waits only if that buffer's copy (STAGE_RING calls back) has not run
        const int k = s->stage_next;
        s->stage_next = (k + 1) % sp_scene::STAGE_RING;
        if (s->tiles_rec[k]) SP_HIP(hipEventSynchronize(s->ev_tiles[k]));
        if ((size_t)n_tiles > s->h_tiles_cap[k]) {
            if (s->h_tiles[k]) (void)hipHostFree(s->h_tiles[k]);
            s->h_tiles[k]     = nullptr;
            s->h_tiles_cap[k] = 0;
            SP_HIP(hipHostMalloc(reinterpret_cast<void**>(&s->h_tiles[k]), (size_t)n_tiles * sizeof(int32_t), hipHostMallocDefault));
            s->h_tiles_cap[k] = (size_t)n_tiles;
        }
        std::memcpy(s->h_tiles[k], p->tile_ids, (size_t)n_tiles * sizeof(int32_t));
        SP_HIP(hipMemcpyAsync(s->d_tiles, s->h_tiles[k], (size_t)n_tiles * sizeof(int32_t), hipMemcpyHostToDevice, stream));
        SP_HIP(hipEventRecord(s->ev_tiles[k], stream));
        s->tiles_rec[k] = true;
        d_ids = s->d_tiles;
    }
    if (s->n_cu == 0) {
        hipDeviceProp_t prop;
        SP_HIP(hipGetDeviceProperties(&prop, s->device));
        s->n_cu = prop.multiProcessorCount;
    }
    const bool timing   = (p->flags & SP_RENDER_STAGE_TIMING) != 0;
    float      stage[4] = { 0, 0, 0, 0 };
    const int  asked    = p->flags & 3;
    int        pipeline = asked;
    if (pipeline == SP_PIPELINE_SAMPLE_CHUNKS && integ != SP_INTEGRATOR_DIRECT_LIGHTING)
        return fail(SP_ERR_UNSUPPORTED, "the sample-chunk pipeline implements DirectLighting");
    const bool wave_ok = integ == SP_INTEGRATOR_DIRECT_LIGHTING && s->dev.n_lights <= spd::WF_MAX_LIGHTS;
    if (pipeline == SP_PIPELINE_WAVEFRONT && !wave_ok)
        return fail(SP_ERR_UNSUPPORTED, "the wavefront pipeline implements DirectLighting (<= 32 lights)");
    // AUTO (measurements: DESIGN.md §3, §6).  The megakernel renders the 1-GPU frame fastest
    // (bunny 1080p @ 256 spp: 2974 Mrays/s, wavefront 2305).  Below SP_CHUNK_MAX_TILES = 24000
    // tiles (the 2-8-GPU shards) one pixel's sample chain bounds the megakernel and the sample
    // chunks win (8-way shard 2444 against 823), when their buffers fit the budget.  With an image
    // light ck_count replays Light::sample, so the chunks pay off only below half that (spheres
    // 1024^2 @ 64 spp, 16384 tiles: chunks 2902, megakernel 2973).  The wavefront runs on request,
    // or from SP_WAVE_MIN_TILES tiles (test hook).
    int64_t wave_min = INT64_MAX, chunk_max = 24000;
    if (const char* v = std::getenv("SP_WAVE_MIN_TILES")) wave_min = std::atoll(v);
    if (const char* v = std::getenv("SP_CHUNK_MAX_TILES")) chunk_max = std::atoll(v);
    const uint32_t spp_u = p->samples_per_pixel;
    int64_t chunks_req = p->chunks_per_pixel;
    if (chunks_req == 0)
        if (const char* v = std::getenv("SP_CHUNKS")) chunks_req = std::max<int64_t>(1, std::atoll(v)); // test hook
    const ChunkPlan cp = chunk_plan(s, n_tiles, spp_u, chunks_req);
    double ck_max_gb = p->chunk_max_gb > 0.0f ? (double)p->chunk_max_gb : 96.0;
    if (p->chunk_max_gb == 0.0f)
        if (const char* v = std::getenv("SP_CHUNK_MAX_GB")) ck_max_gb = std::atof(v); // test hook
    // budget: the caller's cap, and never more than the device can still give (the buffer held
    // from an earlier call is freed first)
    size_t free_b = 0, total_b = 0;
    SP_HIP(hipMemGetInfo(&free_b, &total_b));
    const double ck_budget = std::min(ck_max_gb * 1e9, (double)free_b + (double)s->ck_cap);
    bool image_light = false;
    for (const auto& l : s->host->lights) image_light = image_light || l.kind == SP_LIGHT_IMAGE_ENVIRONMENT;
    // Megakernel tail chunks (below): DirectLighting from 2.5 tiles per persistent wave (16 per CU
    // at full occupancy) and 128 spp, where the draw counts are known from the camera hits.  There
    // the megakernel with its tile order and tail chunks beats the sample chunks (bunny 2-way shard
    // 16200 tiles: 3620-3640 against 3170 Mrays/s, lucy 2-way 3227 against 2885; 3-way, 2.6 tiles
    // per wave: 3398-3412 at a fraction of 0.4 against the fused chunks' 3321-3344; 4-way, 2 per
    // wave: 2820-2980 against 3297 -- profiles/r06/tail/ab_shards*.log, ab_fused*.log).
    // With an image light the preps replay Light::sample (TailArgs::replay): material_spheres with its
    // image light, 1024^2 @ 64 spp (4 tiles per wave), 3814-3826 -> 3890-3895 Mrays/s (ab_spheres.log),
    // so from 64 spp at 4 tiles per wave as well.
    const int64_t tail_waves = (int64_t)std::max(1, s->n_cu) * 16;
    const bool    tail_auto  = integ == SP_INTEGRATOR_DIRECT_LIGHTING && s->dev.n_lights <= 1000 && p->tail_fraction >= 0.0f &&
                           ((spp_u >= 128 && 2 * n_tiles >= 5 * tail_waves) || (spp_u >= 64 && n_tiles >= 4 * tail_waves));
    if (pipeline == SP_PIPELINE_AUTO) {
        if (wave_ok && n_tiles >= wave_min) pipeline = SP_PIPELINE_WAVEFRONT;
        else if (tail_auto) pipeline = SP_PIPELINE_MEGAKERNEL;
        else if (integ == SP_INTEGRATOR_DIRECT_LIGHTING && n_tiles < (image_light ? chunk_max / 2 : chunk_max) &&
                 (double)cp.total <= ck_budget)
            pipeline = SP_PIPELINE_SAMPLE_CHUNKS;
        else pipeline = SP_PIPELINE_MEGAKERNEL; // also when the chunk buffers would not fit the budget
    }
    if (pipeline == SP_PIPELINE_SAMPLE_CHUNKS && cp.total > s->ck_cap) {
        if ((double)cp.total > ck_budget)
            return fail(SP_ERR_UNSUPPORTED, "sample-chunk pipeline: buffers exceed the budget (chunk_max_gb / free "
                                            "device memory; render fewer tiles per call)");
        if (s->ck_buf) (void)hipFree(s->ck_buf);
        s->ck_buf = nullptr;
        s->ck_cap = 0;
        const hipError_t e = hipMalloc(&s->ck_buf, cp.total);
        if (e != hipSuccess) {
            s->ck_buf = nullptr;
            (void)hipGetLastError();
            if (asked != SP_PIPELINE_AUTO) return fail(SP_ERR_HIP, std::string("sample-chunk buffers: ") + hipGetErrorString(e));
            pipeline = SP_PIPELINE_MEGAKERNEL; // AUTO: the megakernel needs no per-sample buffers
        } else {
            s->ck_cap = cp.total;
        }
    }
    SP_HIP(hipMemsetAsync(s->counters, 0, 8 * sizeof(unsigned long long), stream));
    int launches = 0, parts_used = 1;
    int64_t tail_k = 0;  // megakernel tail chunks: tiles cut (tail_ch chunks each)
    int     tail_ch = 0;
    if (pipeline == SP_PIPELINE_WAVEFRONT) {
        const size_t stack_lds = (size_t)4 * s->dev.stack_words * 64 * 4;
        if (stack_lds > 160 * 1024) return fail(SP_ERR_UNSUPPORTED, "BVH too deep for the LDS traversal stack");
        // Pixels in flight per pass: all requested tiles unless the state would exceed the budget
        // (SP_WAVE_MAX_GB, default 64 GB of the 288 GB HBM); larger jobs run in tile chunks.
        double budget_gb = 64.0;
        if (const char* v = std::getenv("SP_WAVE_MAX_GB")) budget_gb = std::atof(v);
        const size_t  per_pix   = spd::wave_bytes_per_pixel(s->dev.n_lights);
        // queue items pack the pixel slot in 27 bits (sp_wave.hip wf_shade)
        const int64_t max_tiles = std::min<int64_t>((int64_t)1 << 21,
                                                    std::max<int64_t>(1, (int64_t)(budget_gb * 1e9 / (double)(per_pix * 64))));
        const int64_t chunk     = std::min<int64_t>(n_tiles, max_tiles);
        const size_t  n         = (size_t)chunk * 64;
        const size_t  need      = n * per_pix + spd::wave_stat_bytes((int64_t)n) + spd::wave_queue_bytes((int64_t)n, s->dev.n_lights) +
                                  n * (size_t)std::max(1, s->dev.n_lights) + 256 * 12;
        if (need > s->wave_cap) {
            if (s->wave_buf) (void)hipFree(s->wave_buf);
            s->wave_buf = nullptr;
            s->wave_cap = 0;
            SP_HIP(hipMalloc(&s->wave_buf, need));
            s->wave_cap = need;
        }
        // carve: every array 256-byte aligned (n is a multiple of 64)
        char* b    = static_cast<char*>(s->wave_buf);
        auto  take = [&](size_t bytes) { char* r = b; b += (bytes + 255) & ~(size_t)255; return r; };
        spd::WaveArgs w{};
        w.n        = (int64_t)n;
        w.tiles_x  = (s->dev.width + 7) / 8;
        w.spp      = p->samples_per_pixel;
        w.mt_state = reinterpret_cast<uint64_t*>(take(n / 64 * 2 * spd::MT_GEN_WORDS * 8));
        w.sh       = reinterpret_cast<float4*>(take(n * (size_t)std::max(1, s->dev.n_lights) * 32));
        w.hit      = reinterpret_cast<float4*>(take(n * 16));
        w.shp      = reinterpret_cast<float4*>(take(n * 16));
        w.acc      = reinterpret_cast<float*>(take(n * 12));
        w.rstate   = reinterpret_cast<uint32_t*>(take(n * 4));
        w.queue    = reinterpret_cast<uint32_t*>(take(spd::wave_queue_bytes((int64_t)n, s->dev.n_lights)));
        w.qcount   = nullptr; // per part (wave_render)
        w.vis      = reinterpret_cast<uint8_t*>(take(n * (size_t)std::max(1, s->dev.n_lights)));
        w.wstat    = reinterpret_cast<unsigned long long*>(take(spd::wave_stat_bytes((int64_t)n)));
        w.counters = s->counters;
        // SP_WAVE_DIAG=<file>: per-wave timeline of one sample's primary + shadow launches
        const char*         diag_path = std::getenv("SP_WAVE_DIAG");
        unsigned long long* d_diag    = nullptr;
        const size_t        diag_n    = 2 * (n / 64) * 4;
        if (diag_path) {
            SP_HIP(hipMalloc(&d_diag, diag_n * 8));
            SP_HIP(hipMemsetAsync(d_diag, 0, diag_n * 8, stream));
        }
        w.diag = d_diag;
        const int per_cu = spd::wave_traverse_blocks_per_cu(s->dev);
        // two halves of the tile list on two streams, their shading kernels alternating (+11 %;
        // 3 or 4 parts measured 1988 / 1821 against 2068 Mrays/s)
        const int n_parts = std::min(2, spd::WF_MAX_PARTS);
        if (!s->ev_fork) {
            SP_HIP(hipEventCreateWithFlags(&s->ev_fork, hipEventDisableTiming));
            for (auto& e : s->ev_shade) SP_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
        }
        for (int k = 0; k + 1 < n_parts; ++k)
            if (!s->aux_stream[k]) {
                SP_HIP(hipStreamCreateWithFlags(&s->aux_stream[k], hipStreamNonBlocking));
                SP_HIP(hipEventCreateWithFlags(&s->ev_join[k], hipEventDisableTiming));
            }
        const size_t n_ev = timing ? 3 * (size_t)w.spp + 3 : 0;
        while (s->stage_ev.size() < n_ev) {
            hipEvent_t e;
            SP_HIP(hipEventCreate(&e));
            s->stage_ev.push_back(e);
        }
        SP_HIP(hipEventRecord(s->ev0, stream));
        for (int64_t t0 = 0; t0 < n_tiles; t0 += chunk) {
            const int64_t nt = std::min<int64_t>(chunk, n_tiles - t0);
            w.n        = nt * 64;
            w.tile_ids = d_ids ? d_ids + t0 : nullptr;
            if (!d_ids && t0 > 0) {
                // identity ids beyond the first chunk: materialise them
                std::vector<int32_t> ids((size_t)nt);
                for (int64_t i = 0; i < nt; ++i) ids[(size_t)i] = (int32_t)(t0 + i);
                if ((size_t)nt > s->d_tiles_cap) {
                    if (s->d_tiles) (void)hipFree(s->d_tiles);
                    s->d_tiles = nullptr;
                    SP_HIP(hipMalloc(&s->d_tiles, (size_t)chunk * sizeof(int32_t)));
                    s->d_tiles_cap = (size_t)chunk;
                }
                SP_HIP(hipMemcpyAsync(s->d_tiles, ids.data(), (size_t)nt * 4, hipMemcpyHostToDevice, stream));
                SP_HIP(hipStreamSynchronize(stream));
                w.tile_ids = s->d_tiles;
            }
            w.pb = 0;
            w.pe = w.n;
            SP_HIP(spd::wave_render(s->dev, w, d_out + (size_t)t0 * 64 * 3, per_cu, s->n_cu, stream,
                                    timing ? s->stage_ev.data() : nullptr, s->aux_stream, n_parts - 1,
                                    s->ev_fork, s->ev_join, s->ev_shade, &parts_used));
            launches += 3 + 4 * (int)w.spp;
            if (d_diag) {
                std::vector<unsigned long long> h(diag_n);
                SP_HIP(hipStreamSynchronize(stream));
                SP_HIP(hipMemcpy(h.data(), d_diag, diag_n * 8, hipMemcpyDeviceToHost));
                if (FILE* f = std::fopen(diag_path, "wb")) {
                    std::fwrite(h.data(), 8, diag_n, f);
                    std::fclose(f);
                }
                (void)hipFree(d_diag);
                d_diag = nullptr;
                w.diag = nullptr;
            }
            if (timing) {
                SP_HIP(hipEventSynchronize(s->stage_ev[n_ev - 1]));
                auto el = [&](size_t a, size_t b) {
                    float ms = 0.0f;
                    (void)hipEventElapsedTime(&ms, s->stage_ev[a], s->stage_ev[b]);
                    return ms;
                };
                stage[0] += el(0, 1) + el(n_ev - 2, n_ev - 1);
                for (uint32_t i = 0; i < w.spp; ++i) {
                    const size_t b = 1 + 3 * (size_t)i;
                    stage[1] += el(b, b + 1);
                    stage[2] += el(b + 1, b + 2);
                    stage[3] += el(b + 2, b + 3);
                }
            }
        }
    } else if (pipeline == SP_PIPELINE_SAMPLE_CHUNKS) {
        // sp_chunk.hip: camera rays for all (pixel, sample) at once, a per-pixel replay of the
        // stream positions into the generator store, then every (tile, chunk) shaded in parallel,
        // and the in-order sum (buffers: chunk_plan above)
        const int    rs_words  = spd::rsqrt_words(s->dev);
        const size_t lds_bytes = (size_t)rs_words * 4 + (size_t)4 * s->dev.stack_words * 64 * 4;
        if (lds_bytes > 160 * 1024) return fail(SP_ERR_UNSUPPORTED, "BVH too deep for the LDS traversal stack");
        const size_t n_px   = (size_t)n_tiles * 64;
        if (!s->ck_ctr) SP_HIP(hipMalloc(&s->ck_ctr, 2 * sizeof(int32_t)));
        const int per_cu = spd::chunk_blocks_per_cu(lds_bytes);
        const int blocks = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)s->n_cu * per_cu, (n_tiles * cp.chunks + 3) / 4));
        char*          base = static_cast<char*>(s->ck_buf);
        spd::ChunkArgs a{};
        a.tile_ids    = d_ids;
        a.num_tiles   = n_tiles;
        a.tiles_x     = (s->dev.width + 7) / 8;
        a.spp         = spp_u;
        a.chunks      = (uint32_t)cp.chunks;
        a.chunk_len   = cp.len;
        a.n_px        = n_px;
        a.hits        = reinterpret_cast<float4*>(base);
        a.L           = reinterpret_cast<float*>(base + cp.b_hits);
        a.gens        = reinterpret_cast<uint64_t*>(base + cp.b_hits + cp.b_L);
        a.gens_per_px = cp.gens;
        a.snap_ctl    = reinterpret_cast<uint32_t*>(base + cp.b_hits + cp.b_L + cp.b_snap);
        a.draws       = cp.known_draws ? reinterpret_cast<uint16_t*>(base + cp.b_hits + cp.b_L + cp.b_snap + cp.b_ctl) : nullptr;
        a.n_lights    = s->dev.n_lights;
        a.counter     = s->ck_ctr;
        a.counters    = s->counters;
        a.out         = d_out;
        // Fused form (known draw counts): ck_camera, then the counts and the shading in ONE persistent
        // queue of the megakernel's tail kernel (sp_mega.hpp, RenderArgs::tail_front): each tile's
        // prep (stream positions, generations into the store) runs P tiles ahead of its chunks, so the
        // HBM-bound twists overlap the shading instead of running as a phase of their own (ck_count).
        // Same store contents and chunk starts, same image.  SP_CK_FUSED=0: the four-kernel form.
        bool fused = cp.known_draws && SP_CK_FUSED;
        if (const char* v = std::getenv("SP_CK_FUSED")) fused = cp.known_draws && std::atoi(v) != 0;
        SP_HIP(hipMemsetAsync(s->ck_ctr, 0, 2 * sizeof(int32_t), stream));
        if (fused) {
            // the tail kernel's LDS (the megakernel's: RSQRTSS table + per-wave stacks) and occupancy
            size_t lds_static = spd::render_static_lds(SP_INTEGRATOR_DIRECT_LIGHTING, 4);
            if (lds_bytes + lds_static > 160 * 1024) fused = false;
        }
        if (fused) {
            const size_t a_hdr = 256, a_rdy = ((size_t)n_tiles * 4 + 255) / 256 * 256, need = a_hdr + 2 * a_rdy;
            if (need > s->tail_cap) {
                if (s->tail_buf) (void)hipFree(s->tail_buf);
                s->tail_buf = nullptr;
                s->tail_cap = 0;
                SP_HIP(hipMalloc(&s->tail_buf, need));
                s->tail_cap = need;
            }
            char*         tb = static_cast<char*>(s->tail_buf);
            spd::TailArgs ta{};
            ta.n_prep      = n_tiles;
            ta.n_items     = n_tiles * cp.chunks;
            ta.chunks      = (uint32_t)cp.chunks;
            ta.chunk_len   = cp.len;
            ta.gens_per_px = cp.gens;
            ta.n_px        = n_px;
            ta.hits        = a.hits;
            ta.L           = a.L;
            ta.gens        = a.gens;
            ta.snap_ctl    = a.snap_ctl;
            ta.draws       = a.draws;
            ta.ready       = reinterpret_cast<uint32_t*>(tb + a_hdr);
            // the camera pass as the queue's first items (SP_CK_CAMFOLD; blocks of SP_CK_CAM_BLOCK
            // samples per item) instead of the ck_camera kernel before it
            bool cam_fold = SP_CK_CAMFOLD;
            if (const char* v = std::getenv("SP_CK_CAMFOLD")) cam_fold = std::atoi(v) != 0;
            if (cam_fold) {
                ta.cam_block = SP_CK_CAM_BLOCK;
                if (const char* v = std::getenv("SP_CK_CAM_BLOCK")) ta.cam_block = (uint32_t)std::max(1, std::atoi(v));
                ta.n_cam     = n_tiles * (int64_t)((spp_u + ta.cam_block - 1) / ta.cam_block);
                ta.cam_done  = reinterpret_cast<uint32_t*>(tb + a_hdr + a_rdy);
                ta.draws_out = a.draws;
            }
            SP_HIP(hipMemcpyAsync(tb, &ta, sizeof(ta), hipMemcpyHostToDevice, stream));
            SP_HIP(hipMemsetAsync(ta.ready, 0, 2 * a_rdy, stream));
            spd::RenderArgs ra{};
            ra.out          = d_out;
            ra.tile_ids     = d_ids;
            ra.num_tiles    = n_tiles;
            ra.tiles_x      = a.tiles_x;
            ra.spp          = spp_u;
            ra.integrator   = integ;
            ra.tile_counter = s->ck_ctr;
            ra.counters     = s->counters;
            ra.tail_prep    = ta.n_prep;
            ra.tail_items   = ta.n_items;
            const int     t_per_cu = spd::tail_blocks_per_cu(0, lds_bytes); // 0: sp_fused_kernel
            const int64_t t_waves  = (int64_t)s->n_cu * t_per_cu * 4;
            // P: the preps ahead of the first chunks; the rest are dealt one per tile's chunks
            int64_t front = std::max<int64_t>(1, t_waves / SP_CK_FRONT_DIV);
            if (const char* v = std::getenv("SP_CK_FRONT_DIV")) front = std::max<int64_t>(1, t_waves / std::max(1, std::atoi(v)));
            ra.tail_front = front;
            ra.tail_cam   = ta.n_cam;
            ra.tail       = reinterpret_cast<const spd::TailArgs*>(tb);
            const int t_blocks = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)s->n_cu * t_per_cu,
                                                                               (n_tiles * (cp.chunks + 1) + 3) / 4));
            SP_HIP(hipEventRecord(s->ev0, stream));
            if (!cam_fold) SP_HIP(spd::chunk_camera(s->dev, a, s->n_cu, stream));
            SP_HIP(spd::launch_tail(s->dev, ra, 0, t_blocks, lds_bytes, stream));
            SP_HIP(spd::chunk_sum(s->dev, a, stream));
            launches = cam_fold ? 2 : 3;
        } else {
            SP_HIP(hipEventRecord(s->ev0, stream));
            SP_HIP(spd::chunk_render(s->dev, a, blocks, s->n_cu, stream));
            launches = 4;
        }
    } else {
        const int    rs_words  = spd::rsqrt_words(s->dev);
        const size_t lds_bytes = (size_t)rs_words * 4 + (size_t)4 * s->dev.stack_words * 64 * 4;
        // the kernel's static LDS counts too (the largest over the variants this call may pick)
        size_t lds_static = 0;
        for (int v = 2; v <= 4; ++v) lds_static = std::max(lds_static, spd::render_static_lds(integ, v));
        const size_t lds_all = lds_bytes + lds_static;
        if (lds_all > 160 * 1024) return fail(SP_ERR_UNSUPPORTED, "BVH too deep for the LDS traversal stack");
        // waves per SIMD the kernel is compiled for (SP_KERNEL_VARIANT): DirectLighting 4,
        // IterativeRRNEE 3 -- but never more than the LDS lets run (one 4-wave block per wave per
        // SIMD): a deep BVH's stacks (lucy: 3 blocks per CU) would leave the extra occupancy's
        // register budget paid for in spills and unused (lucy 1080p @ 256 spp: 2007 Mrays/s at 3
        // waves, 1879 at 4; profiles/r02/s5)
        const int lds_waves = (int)std::min<size_t>(8, (160 * 1024) / lds_all);
        int       variant   = integ == SP_INTEGRATOR_ITERATIVE_RRNEE ? 3 : 4;
        variant             = std::max(2, std::min(variant, lds_waves));
        if (waves_req) variant = waves_req;
        const int     per_cu  = spd::render_blocks_per_cu(integ, variant, lds_bytes);
        const int64_t max_blk = (int64_t)s->n_cu * per_cu;
        const int64_t need    = (n_tiles + 3) / 4;
        const int     blocks  = (int)std::max<int64_t>(1, std::min(max_blk, need));
        const size_t  waves   = (size_t)blocks * 4;
        if (waves > s->mt_waves) {
            if (s->mt_state) (void)hipFree(s->mt_state);
            s->mt_state = nullptr;
            SP_HIP(hipMalloc(&s->mt_state, waves * 2 * (size_t)spd::MT_GEN_WORDS * sizeof(uint64_t)));
            s->mt_waves = waves;
        }
        SP_HIP(hipMemsetAsync(s->tile_counter, 0, sizeof(int32_t), stream));
        spd::Scene sc_run    = s->dev; // the resident scene with this render's options
        sc_run.merge_queries = (p->flags & SP_RENDER_PER_LANE_QUERIES) ? 0 : 1;
        spd::RenderArgs a{};
        a.out          = d_out;
        a.tile_ids     = d_ids;
        a.num_tiles    = n_tiles;
        a.tiles_x      = (s->dev.width + 7) / 8;
        a.spp          = p->samples_per_pixel;
        a.integrator   = integ;
        a.tile_counter = s->tile_counter;
        a.mt_state     = s->mt_state;
        a.counters     = s->counters;
        // BruteForce / Whitted recursion deeper than the in-register arrays: global level records
        a.deep        = nullptr;
        a.deep_stride = 0;
        if ((integ == SP_INTEGRATOR_BRUTE_FORCE || integ == SP_INTEGRATOR_WHITTED) && s->dev.max_depth > MAX_RECURSION) {
            const size_t lanes = waves * 64; // persistent waves of this launch (4 per block)
            const size_t bytes = lanes * ((size_t)s->dev.max_depth + 1) * 5 * sizeof(float);
            if (bytes > s->deep_cap) {
                if (s->deep_buf) (void)hipFree(s->deep_buf);
                s->deep_buf = nullptr;
                s->deep_cap = 0;
                SP_HIP(hipMalloc(&s->deep_buf, bytes));
                s->deep_cap = bytes;
            }
            a.deep        = static_cast<float*>(s->deep_buf);
            a.deep_stride = lanes;
        }
        SP_HIP(hipEventRecord(s->ev0, stream));
        // SP_TILE_DIAG=<file>: per-tile timeline {t0, t1, wave, item} (u64, s_memrealtime 100 MHz) and,
        // in a -DSP_MEGA_PROF build, shader clocks in trace / light sample / eval / occlusion
        const char*         tdiag_path = std::getenv("SP_TILE_DIAG");
        unsigned long long* tdiag      = nullptr;
        if (tdiag_path) {
            // the -DSP_WAVE_PROF / -DSP_TRAFFIC_DIAG builds add their totals into words 0..47
            const size_t words = std::max<size_t>((size_t)n_tiles * 8, 48);
            SP_HIP(hipMalloc(&tdiag, words * sizeof(unsigned long long)));
            SP_HIP(hipMemsetAsync(tdiag, 0, words * sizeof(unsigned long long), stream));
        }
        a.tile_diag = tdiag;
        a.order     = nullptr;
        a.tile_time = nullptr;
        // Tile order (sp_mega.hip tile_order): a one-sample probe pass times every tile, and the
        // queue is ordered by cost class (slower than `hoist` x the mean first, the cheapest last),
        // so the frame does not end with a few waves finishing expensive tiles alone.  Part of the
        // render (timed with it); stream-ordered, no host wait.  Used where it measured faster
        // (profiles/r03/ab_tile_order.txt, profiles/r04/tile_classes/): DirectLighting with many
        // tiles per persistent wave and a probe that costs little of the frame (bunny 1080p @ 256
        // spp, 7.9 tiles per wave; lucy; spheres 1024^2 @ 64 spp, 4 tiles per wave, loses 1 %);
        // IterativeRRNEE, whose tile costs spread wider (paths end at any depth), from 4 tiles per
        // wave and 16 spp (elf 1024^2 @ 16 spp +1.7 %; elf's 8-way shard +3 % with two classes, +5 % more with six).  DirectLighting and
        // IterativeRRNEE have probe kernels (sp_probe_*.hip); the other integrators render in queue
        // order.  sp_render_params.tile_order_factor > 0 forces it with that factor, < 0 turns it off.
        const bool rrnee = integ == SP_INTEGRATOR_ITERATIVE_RRNEE;
        // (DirectLighting with tail chunks: from 3 tiles per wave, tail_auto above)
        float hoist = (n_tiles >= (rrnee ? 4 : 6) * (int64_t)waves && p->samples_per_pixel >= (rrnee ? 16u : 128u)) ? 2.0f : 0.0f;
        if (tail_auto && 2 * n_tiles >= 5 * (int64_t)waves) hoist = 2.0f; // the tail chunks need the order
        if (p->tile_order_factor != 0.0f) hoist = std::max(0.0f, p->tile_order_factor);
        if (hoist > 0.0f && n_tiles > (int64_t)waves && spd::has_probe(integ)) {
            if ((size_t)n_tiles > s->order_cap) {
                if (s->d_tile_time) (void)hipFree(s->d_tile_time);
                if (s->d_order) (void)hipFree(s->d_order);
                s->d_tile_time = nullptr;
                s->d_order     = nullptr;
                s->order_cap   = 0;
                SP_HIP(hipMalloc(&s->d_tile_time, (size_t)n_tiles * sizeof(float)));
                SP_HIP(hipMalloc(&s->d_order, (size_t)n_tiles * sizeof(int32_t)));
                s->order_cap = (size_t)n_tiles;
            }
            if (!s->probe_counters) SP_HIP(hipMalloc(&s->probe_counters, 8 * sizeof(unsigned long long)));
            spd::RenderArgs pr = a;
            pr.spp       = 1; // 2 or 4 probe samples measured no better (profiles/r03/ab_tile_order.txt, r04/tile_classes)
            pr.tile_time = s->d_tile_time;
            pr.counters  = s->probe_counters; // the probe's rays are not the render's
            pr.tile_diag = nullptr;
            // every 2nd slot timed where tail chunks follow and a wave takes 6 tiles or more (the others
            // interpolated by the order kernel: bunny +0.25 %, lucy +0.2 %); at 4 tiles per wave the
            // 2-way shard lost 2.5 % with it (spheres gained 0.6-0.8 %), and IterativeRRNEE, whose order
            // has no tail chunks behind it, lost 2-4 % on elf's shard (profiles/r06/tail/ab_probe_step*.log)
            pr.probe_step = (integ == SP_INTEGRATOR_DIRECT_LIGHTING && (tail_auto || p->tail_fraction > 0.0f) &&
                             n_tiles >= 6 * (int64_t)waves) ? 2 : 1;
            if (const char* v = std::getenv("SP_PROBE_STEP")) pr.probe_step = std::max(1, std::atoi(v));
            SP_HIP(spd::launch_probe(sc_run, pr, integ, variant, blocks, lds_bytes, stream));
            // cost estimates blended with their queue neighbours only where those sit at known
            // image offsets: a whole frame, or a host list with a constant stride (the bench's list,
            // a rank's interleaved shard; order_neighbours); any other list keeps each tile's own time
            SP_HIP(spd::launch_tile_order(s->d_tile_time, n_tiles, hoist, order_neighbours(p, listed, n_tiles, a.tiles_x),
                                          pr.probe_step, s->d_order, stream));
            SP_HIP(hipMemsetAsync(s->tile_counter, 0, sizeof(int32_t), stream));
            a.order = s->d_order;
            launches += 2;
        }
        // Tail chunks (sp_mega.hpp, sp_device.hpp TailArgs): the K = tail_frac x n_tiles most
        // expensive tiles of the order are rendered as sample chunks at the end of the queue.
        // DirectLighting at 3 or 4 waves per SIMD with the tile order; the preps take the draw counts
        // from the camera hits, or with an image light replay Light::sample on the stream (TailArgs
        // replay); SP_TAIL_FRAC (0: off) and SP_TAIL_CHUNKS override.
        spd::ChunkArgs tail_sum{};
        // counts replayed on the stream (an image light, or SP_CHUNK_REPLAY): the 4-wave kernel only
        const bool tail_replay = !chunk_plan(s, 1, spp_u, 1).known_draws;
        if (integ == SP_INTEGRATOR_DIRECT_LIGHTING && (variant == 4 || (variant == 3 && !tail_replay)) && a.order) {
            // automatic: SP_TAIL_FRAC, or the environment's SP_TAIL_FRAC (A/B runs); the caller's
            // tail_fraction when set (< 0: off)
            // automatic: one tile per persistent wave's worth (waves / n_tiles: 0.126 for the 1-GPU
            // 1080p frame, 0.25 for a 2-way shard, 0.38 for a 3-way one), within [SP_TAIL_FRAC, 0.4]
            // -- measured best 0.12-0.16, 0.2-0.3 and 0.4 there (profiles/r06/tail/)
            float tail_frac = std::min(0.4f, std::max(SP_TAIL_FRAC, (float)((double)waves / (double)n_tiles)));
            tail_ch         = SP_TAIL_CHUNKS;
            if (const char* v = std::getenv("SP_TAIL_FRAC")) tail_frac = (float)std::atof(v);
            if (const char* v = std::getenv("SP_TAIL_CHUNKS")) tail_ch = std::atoi(v);
            if (p->tail_fraction != 0.0f) tail_frac = p->tail_fraction;
            const ChunkPlan tp = chunk_plan(s, 1, spp_u, std::max(1, tail_ch));
            if (tail_frac > 0.0f) {
                // ceil(frac x n), with frac the f32 caller value (0.05f x 5120 = 256.0000038: 256 tiles)
                tail_k = std::min<int64_t>(n_tiles, std::max<int64_t>(1, (int64_t)std::ceil((double)tail_frac * (double)n_tiles - 1e-3)));
                const ChunkPlan cp    = chunk_plan(s, tail_k, spp_u, std::max(1, tail_ch));
                const size_t    a_hdr = 256, a_rdy = ((size_t)tail_k * 4 + 255) / 256 * 256;
                const size_t    need  = a_hdr + a_rdy + cp.b_hits + cp.b_L + cp.b_snap + cp.b_ctl;
                // the sample chunks' budget (chunk_max_gb, never more than the device can still give):
                // 20 GB for bunny's 4096 tail tiles (the store: 30 generations per pixel); a scene
                // with many lights (a store bound of 34 draws per light and sample) renders without
                // tail chunks rather than fail
                const double tail_budget = std::min(ck_max_gb * 1e9, (double)free_b + (double)s->tail_cap);
                if ((double)need > tail_budget) tail_k = 0;
                if (tail_k > 0 && need > s->tail_cap) {
                    if (s->tail_buf) (void)hipFree(s->tail_buf);
                    s->tail_buf = nullptr;
                    s->tail_cap = 0;
                    if (hipMalloc(&s->tail_buf, need) != hipSuccess) {
                        s->tail_buf = nullptr;
                        (void)hipGetLastError();
                        tail_k = 0;
                    } else {
                        s->tail_cap = need;
                    }
                }
            }
            if (tail_k > 0) {
                const ChunkPlan cp    = chunk_plan(s, tail_k, spp_u, std::max(1, tail_ch));
                const size_t    a_hdr = 256, a_rdy = ((size_t)tail_k * 4 + 255) / 256 * 256;
                char*         base = static_cast<char*>(s->tail_buf);
                spd::TailArgs ta{};
                tail_ch        = (int)cp.chunks;
                ta.n_prep      = tail_k;
                ta.replay      = tail_replay ? 1 : 0; // an image light: the preps replay Light::sample
                ta.n_items     = tail_k * cp.chunks;
                ta.chunks      = (uint32_t)cp.chunks;
                ta.chunk_len   = cp.len;
                ta.gens_per_px = cp.gens;
                ta.n_px        = (size_t)tail_k * 64;
                ta.ready       = reinterpret_cast<uint32_t*>(base + a_hdr);
                ta.hits        = reinterpret_cast<float4*>(base + a_hdr + a_rdy);
                ta.L           = reinterpret_cast<float*>(base + a_hdr + a_rdy + cp.b_hits);
                ta.gens        = reinterpret_cast<uint64_t*>(base + a_hdr + a_rdy + cp.b_hits + cp.b_L);
                ta.snap_ctl    = reinterpret_cast<uint32_t*>(base + a_hdr + a_rdy + cp.b_hits + cp.b_L + cp.b_snap);
                // the kernel reads TailArgs from device memory (stream-ordered behind the previous
                // call's kernels, which may still read it)
                SP_HIP(hipMemcpyAsync(base, &ta, sizeof(ta), hipMemcpyHostToDevice, stream));
                SP_HIP(hipMemsetAsync(ta.ready, 0, (size_t)tail_k * 4, stream));
                a.tail_prep  = ta.n_prep;
                a.tail_items = ta.n_items;
                a.tail       = reinterpret_cast<const spd::TailArgs*>(base);
                tail_sum.tile_ids  = d_ids;
                tail_sum.num_tiles = tail_k;
                tail_sum.tiles_x   = a.tiles_x;
                tail_sum.spp       = spp_u;
                tail_sum.n_px      = ta.n_px;
                tail_sum.L         = ta.L;
                tail_sum.out       = d_out;
                tail_sum.slot_map  = s->d_order; // chunk slot k is queue item k: tile slot order[k]
            }
        }
        if (timing) {
            if (!s->ev_render) SP_HIP(hipEventCreate(&s->ev_render));
            SP_HIP(hipEventRecord(s->ev_render, stream));
        }
        if (tail_k > 0) {
            const int     t_var    = tail_replay ? -variant : variant; // -4: the replaying tail kernel
            const int     t_per_cu = spd::tail_blocks_per_cu(t_var, lds_bytes);
            const int64_t t_need   = (n_tiles + a.tail_items + 3) / 4;
            const int     t_blocks = (int)std::max<int64_t>(1, std::min<int64_t>((int64_t)s->n_cu * t_per_cu, t_need));
            SP_HIP(spd::launch_tail(sc_run, a, t_var, t_blocks, lds_bytes, stream));
            SP_HIP(spd::chunk_sum(sc_run, tail_sum, stream));
            launches += 1;
        } else {
            SP_HIP(spd::launch_render(sc_run, a, integ, variant, blocks, lds_bytes, stream));
        }
        if (tdiag) { // diagnostic: waits for the render
            SP_HIP(hipStreamSynchronize(stream));
            std::vector<unsigned long long> rec((size_t)n_tiles * 8);
            SP_HIP(hipMemcpy(rec.data(), tdiag, rec.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
            (void)hipFree(tdiag);
            if (FILE* f = std::fopen(tdiag_path, "wb")) {
                std::fwrite(rec.data(), sizeof(unsigned long long), rec.size(), f);
                std::fclose(f);
            }
        }
        launches += 1;
    }
    SP_HIP(hipEventRecord(s->ev1, stream));
    SP_HIP(hipEventRecord(s->ev_done, stream));
    s->done_rec = true;
    // stream order: without stats nothing waits -- the render is only enqueued
    if (stats) {
        SP_HIP(hipEventSynchronize(s->ev1));
        unsigned long long c[8];
        SP_HIP(hipMemcpy(c, s->counters, sizeof(c), hipMemcpyDeviceToHost));
        float ms = 0.0f;
        SP_HIP(hipEventElapsedTime(&ms, s->ev0, s->ev1));
        if (pipeline == SP_PIPELINE_SAMPLE_CHUNKS) {
            // camera rays and samples: one per inside pixel and sample (counted here, not on device)
            std::vector<int32_t> ids;
            if (listed) {
                ids.resize((size_t)n_tiles);
                if (p->tile_ids) std::memcpy(ids.data(), p->tile_ids, ids.size() * sizeof(int32_t));
                else SP_HIP(hipMemcpy(ids.data(), p->d_tile_ids, ids.size() * sizeof(int32_t), hipMemcpyDeviceToHost));
            }
            int64_t       inside = 0;
            const int32_t tw     = (s->dev.width + 7) / 8;
            for (int64_t sl = 0; sl < n_tiles; ++sl) {
                const int64_t t = listed ? ids[(size_t)sl] : sl;
                if (t < 0 || t >= total) continue;
                const int64_t x0 = (t % tw) * 8, y0 = (t / tw) * 8;
                inside += std::min<int64_t>(8, s->dev.width - x0) * std::min<int64_t>(8, s->dev.height - y0);
            }
            c[0] = (s->dev.max_depth > 0 ? (unsigned long long)inside * spp_u : 0ull) + c[1];
            c[2] = (unsigned long long)inside * spp_u;
        }
        stats->rays        = c[0];
        stats->shadow_rays = c[1];
        stats->samples     = c[2];
        stats->rng_draws   = c[3];
        stats->kernel_ms   = ms;
        stats->pipeline    = pipeline;
        stats->launches    = launches;
        stats->primary_hits = c[4];
        stats->parts        = parts_used;
        stats->stack_depth  = s->dev.stack_depth;
        stats->tail_tiles   = (int32_t)tail_k;
        stats->tail_chunks  = tail_k > 0 ? tail_ch : 0;
        if (pipeline == SP_PIPELINE_MEGAKERNEL && timing) { // [0] the render kernel, [1] probe + tile order
            float r = ms;
            if (s->ev_render) SP_HIP(hipEventElapsedTime(&r, s->ev_render, s->ev1));
            stage[0] = r;
            stage[1] = ms - r;
        }
        for (int k = 0; k < 4; ++k) stats->stage_ms[k] = stage[k];
    }
    return SP_OK;
}

int sp_render_tiles_host(sp_scene* s, const sp_render_params* p, float* h_out, sp_render_stats* stats)
{
    if (!s || !p || !h_out) return fail(SP_ERR_ARG, "null argument");
    if (s->device < 0) return fail(SP_ERR_STATE, "sp_scene_upload must be called before rendering");
    SP_HIP(hipSetDevice(s->device));
    int64_t total;
    sp_tile_count(s->dev.width, s->dev.height, &total);
    const int64_t n     = p->tile_ids ? p->num_tiles : total;
    const size_t  bytes = (size_t)std::max<int64_t>(n, 1) * 64 * 3 * sizeof(float);
    float*        d     = nullptr;
    SP_HIP(hipMalloc(&d, bytes));
    int rc = sp_render_tiles(s, p, d, stats);
    if (rc == SP_OK) {
        hipError_t e = hipMemcpy(h_out, d, (size_t)n * 64 * 3 * sizeof(float), hipMemcpyDeviceToHost);
        if (e != hipSuccess) rc = fail(SP_ERR_HIP, hipGetErrorString(e));
    }
    (void)hipFree(d);
    return rc;
}

int sp_tiles_to_image(int32_t width, int32_t height, const int32_t* tile_ids, int64_t num_tiles, const float* tiles,
                      float* image)
{
    if (!tiles || !image || width <= 0 || height <= 0) return fail(SP_ERR_ARG, "bad argument");
    int64_t total;
    sp_tile_count(width, height, &total);
    const int64_t n  = tile_ids ? num_tiles : total;
    const int32_t tw = (width + 7) / 8;
    for (int64_t sl = 0; sl < n; ++sl) {
        const int64_t t = tile_ids ? tile_ids[sl] : sl;
        if (t < 0 || t >= total) return fail(SP_ERR_ARG, "tile id out of range");
        const int32_t x0 = (int32_t)(t % tw) * 8, y0 = (int32_t)(t / tw) * 8;
        for (uint32_t m = 0; m < 64; ++m) {
            uint32_t a = m & 0x55u, b = (m >> 1) & 0x55u;
            a = (a | (a >> 1)) & 0x33u; a = (a | (a >> 2)) & 0x0fu;
            b = (b | (b >> 1)) & 0x33u; b = (b | (b >> 2)) & 0x0fu;
            const int32_t x = x0 + (int32_t)a, y = y0 + (int32_t)b;
            if (x >= width || y >= height) continue;
            for (int c = 0; c < 3; ++c) image[((size_t)y * width + x) * 3 + c] = tiles[((size_t)sl * 64 + m) * 3 + c];
        }
    }
    return SP_OK;
}

int sp_write_pfm(const char* path, int32_t width, int32_t height, const float* image)
{
    if (!path || !image) return fail(SP_ERR_ARG, "null argument");
    FILE* f = std::fopen(path, "wb");
    if (!f) return fail(SP_ERR_IO, std::string("Unable to open ") + path);
    std::fprintf(f, "PF\n%d %d\n%d\n", width, height, -1);
    for (int32_t j = height - 1; j >= 0; --j)
        std::fwrite(image + (size_t)j * width * 3, sizeof(float), (size_t)width * 3, f);
    std::fclose(f);
    return SP_OK;
}

int sp_scene_bvh_build_info(const sp_scene* s, int32_t bvh_mode, sp_bvh_info* out)
{
    if (!s || !out) return fail(SP_ERR_ARG, "null argument");
    if (bvh_mode != 0 && bvh_mode != 1) return fail(SP_ERR_ARG, "bvh_mode must be 0 (SAH) or 1 (reference)");
    try {
        const sph::Scene&    h = *s->host;
        std::vector<int32_t> prims;
        size_t               part = 0;
        sp_upload_params up{};
        up.bvh_mode = bvh_mode;
        UploadOpts opts;
        if (int rc0 = resolve_upload(&up, opts)) return rc0;
        const sph::Bvh       bvh  = geometry_bvh(h, opts, prims, part);
        *out                      = sp_bvh_info{};
        out->depth                = bvh.max_depth;
        out->nodes                = (int64_t)bvh.nodes.size();
        out->slots                = (int64_t)bvh.prim_order.size();
        std::vector<int32_t> lids;
        size_t               lpart = 0;
        out->light_depth           = light_bvh(h, lids, lpart).max_depth;
        const bool stackless       = stackless_for(opts, std::max(out->depth, out->light_depth));
        if (wide_enabled(opts) && !bvh.nodes.empty() && !stackless) out->wide_depth = sph::build_wide(bvh).depth;
        out->stack_depth = stackless ? 0 : stack_entries(out->depth, out->wide_depth, out->light_depth,
                                                          out->wide_depth && opts.wide_closest);
        return SP_OK;
    } catch (const std::exception& e) {
        return fail(SP_ERR_UNSUPPORTED, std::string("BVH build failed: ") + e.what());
    }
}

int sp_scene_device_bytes(const sp_scene* s, int64_t* bytes)
{
    if (!s || !bytes || s->device < 0) return fail(SP_ERR_STATE, "scene not uploaded");
    int64_t b = 0;
    for (const auto& d : s->bufs) b += (int64_t)d.bytes;
    *bytes = b;
    return SP_OK;
}

int sp_scene_bvh_info(const sp_scene* s, int32_t* depth, int64_t* nodes, int64_t* slots)
{
    if (!s || s->device < 0) return fail(SP_ERR_STATE, "scene not uploaded");
    if (depth) *depth = s->geom_depth;
    if (nodes) *nodes = (int64_t)s->geom_nodes;
    if (slots) *slots = (int64_t)s->geom_slots;
    return SP_OK;
}

} // extern "C"
