// sp_wpath.hip -- wavefront form of the multi-bounce iterative integrators:
// BruteForceIntegratorIterative (Integrators/Integrator.cpp:160), BruteForceIntegratorIterativeRR
// (:211) and IntegratorIterativeRRNEE (:550, with estimate_direct_mis :486).
//
// The megakernel (sp_mega.hpp) runs a pixel's samples in a lane, in lock step with the other 63
// lanes of its tile: a wave waits for its longest path at every sample, and it carries the
// shading kernel's registers through every traversal step.  Here each path is cut at its ray
// queries and the two halves run as separate kernels over a pool of tile slots:
//
//   wp_trace  one query per unfinished pixel: extension (intersect_lights + intersect), shadow
//             (intersect_p) or MIS (intersect_lights + intersect_p) -- traversal only, small
//             register footprint, LDS stack
//   wp_shade  consumes the query's result and advances the pixel's path to its next query:
//             material sampling, light sampling and evaluation (every RNG draw, in reference
//             order), throughput and Russian roulette; a finished path adds to the pixel's sum
//             and the next sample's camera ray is issued at once, so the lanes of a tile run
//             their samples independently; a finished pixel writes its output, and when all
//             64 pixels of a slot are done the slot takes the next tile from the caller's list
//             (TileScheduler::get_next_tile, one atomic per tile)
//
// Host loop: (wp_trace, wp_shade) pairs until the active-slot counter reaches zero (polled
// every WP_POLL iterations with a lag, so the host never waits on the GPU in the loop).
//
// Per pixel the floating-point sequence and the RNG draw order are exactly the megakernel's
// (same device functions, same accumulation order), so the two pipelines are bit-identical
// (tests/test_gpu_parity.py).
//
// HBM layout: S slots x 64 lanes = n pixel states; per state SoA float4 fields F_* below
// (ps[field * n + p]), phase/rstate/sample/depth words, and the mt19937_64 state of the slot
// ([slot][buf][312][64] u64 as in the other pipelines).
#include "sp_wave.hpp"
#include "sp_path.hpp"

#include <algorithm>
#include <cstdlib>
#include <vector>

namespace spd {

namespace {

constexpr int WP_BLOCK = 256; // 4 waves = 4 slots per block
constexpr int WP_POLL  = 16;

// pixel phases (low byte of phase[p]; bits 8.. hold the NEE light index)
enum : uint32_t { PH_EXT = 0, PH_SHADOW = 1, PH_MIS = 2, PH_DONE = 3 };

// state fields, float4 each
enum {
    F_L  = 0,  // L.rgb, thr.r
    F_T  = 1,  // thr.g, thr.b, material (bits), s.pdf
    F_P  = 2,  // shading point p.xyz (== ray_at(ray, t), the next ray's origin), ls.pdf
    F_N  = 3,  // n.xyz, ms.pdf
    F_WO = 4,  // wo.xyz, MIS weight
    F_SD = 5,  // bounce sample direction xyz, -
    F_SC = 6,  // bounce sample color rgb, -
    F_LS = 7,  // light sample L rgb, -
    F_LR = 8,  // estimate_direct_mis partial sum rgb, -
    F_MC = 9,  // MIS material sample color rgb, -
    F_Q0 = 10, // query origin xyz, tmin
    F_Q1 = 11, // query direction xyz, tmax
    F_H  = 12, // closest hit {t, code, beta, gamma}
    F_LH = 13, // light hit {L.rgb, flags: 1 hit | 2 occluded | (env + 1) << 2}
    NF   = 14
};

struct PathArgs {
    int64_t             n;          // slots * 64
    int32_t             slots;
    const int32_t*      tile_ids;   // caller's tile list (nullptr: identity)
    int64_t             num_tiles;
    int32_t             tiles_x;
    uint32_t            spp;
    float*              out;        // tile-packed, caller slot = position in the tile list
    int32_t*            next_tile;  // [1] next tile position to hand out
    int32_t*            active;     // [1] slots still holding a tile
    int32_t*            slot_tile;  // [slots] tile position held by the slot, -1 = none
    uint32_t*           phase;      // [n]
    uint32_t*           rstate;     // [n]
    uint32_t*           sample;     // [n] current sample index
    uint32_t*           depth;      // [n]
    float*              acc;        // [3][n]
    float4*             ps;         // [NF][n]
    uint64_t*           mt_state;   // [slots][2][312][64]
    unsigned long long* wstat;      // [slots][ST_N]
};

enum { ST_RAYS = 0, ST_SHADOW = 1, ST_SAMPLES = 2, ST_DRAWS = 3, ST_N = 4 };

__device__ __forceinline__ void slot_count(unsigned long long* slot, int k, uint32_t v)
{
    uint32_t s = v;
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
    if ((threadIdx.x & 63) == 0 && s) slot[k] += s;
}

__device__ __forceinline__ float4& F(const PathArgs& a, int f, int64_t p) { return a.ps[(size_t)f * a.n + p]; }

__device__ __forceinline__ Rng rng_load(const PathArgs& a, int64_t p)
{
    Rng            r;
    const uint32_t st = a.rstate[p];
    r.base  = a.mt_state + (size_t)(p >> 6) * (2 * MT_N * 64) + (p & 63);
    r.idx   = (int)(st & 0xffffu);
    r.cur   = (int)((st >> 16) & 1u);
    r.ready = (int)((st >> 17) & 1u);
    r.draws = 0;
    return r;
}
__device__ __forceinline__ void rng_store(const PathArgs& a, int64_t p, const Rng& r)
{
    a.rstate[p] = (uint32_t)r.idx | ((uint32_t)r.cur << 16) | ((uint32_t)r.ready << 17);
}

struct Pix {
    uint32_t px, py;
    bool     inside;
};
__device__ __forceinline__ Pix pixel_of(const Scene& sc, const PathArgs& a, int32_t pos, uint32_t lane)
{
    const int32_t tile = a.tile_ids ? a.tile_ids[pos] : pos;
    Pix           r;
    r.px     = (uint32_t)((tile % a.tiles_x) * 8) + morton_decode_1(lane);
    r.py     = (uint32_t)((tile / a.tiles_x) * 8) + morton_decode_1(lane >> 1);
    r.inside = (int)r.px < sc.width && (int)r.py < sc.height;
    return r;
}

// RSequenceSampler::get_next_2D + PerspectiveCamera::generate_ray (main.cpp:95-97)
__device__ __forceinline__ Ray camera_ray(const Scene& sc, const Pix& pr, uint32_t i, const Rsq& q)
{
    const uint32_t seed2d = ((pr.px << 16u) | pr.py) ^ 0x6184faf4u;
    const float    sx     = rseq_component(seed2d, sc.alpha2_0, i);
    const float    sy     = rseq_component(seed2d, sc.alpha2_1, i);
    const float    fx     = (float)(int)pr.px + sx;
    const float    fy     = (float)(int)pr.py + sy;
    Ray            ray;
    ray.o = sc.camera.p;
    ray.d = normalize(add(add(scale(fx, sc.camera.vx), scale(fy, sc.camera.vy)), sc.camera.vz), q);
    return ray;
}

__device__ __forceinline__ void put_query(const PathArgs& a, int64_t p, const Ray& r, float tmin, float tmax)
{
    F(a, F_Q0, p) = make_float4(r.o.x, r.o.y, r.o.z, tmin);
    F(a, F_Q1, p) = make_float4(r.d.x, r.d.y, r.d.z, tmax);
}

// Start sample `i` of a pixel whose RNG is already positioned: L = 0, throughput = 1, depth 0,
// camera ray as the first extension query.  Returns false when the path makes no query at all
// (max_depth <= 0): its L = 0 is added by the caller.
__device__ __forceinline__ bool start_sample(const Scene& sc, const PathArgs& a, int64_t p, const Pix& pr, uint32_t i,
                                             const Rsq& q)
{
    if (sc.max_depth <= 0) return false;
    const Ray ray = camera_ray(sc, pr, i, q);
    put_query(a, p, ray, k_ray_epsilon, k_infinite);
    F(a, F_L, p) = make_float4(0.0f, 0.0f, 0.0f, 1.0f);
    float4 t     = F(a, F_T, p);
    t.x = 1.0f;
    t.y = 1.0f;
    F(a, F_T, p) = t;
    a.depth[p]   = 0;
    a.phase[p]   = PH_EXT;
    return true;
}

// Assign tile position `pos` to slot `slot` (called by all 64 lanes of the slot's wave): seed
// every pixel's mt19937_64 (get_integrator_sampler, main.cpp:73), zero its sum and issue sample 0.
__device__ void slot_begin(const Scene& sc, const PathArgs& a, int32_t slot, int32_t pos, const Rsq& q)
{
    const uint32_t lane = threadIdx.x & 63u;
    const int64_t  p    = (int64_t)slot * 64 + lane;
    const Pix      pr   = pixel_of(sc, a, pos, lane);
    a.acc[p]            = 0.0f;
    a.acc[a.n + p]      = 0.0f;
    a.acc[2 * a.n + p]  = 0.0f;
    a.sample[p]         = 0;
    a.phase[p]          = PH_DONE;
    uint32_t samples    = 0;
    float*   o          = a.out + ((size_t)pos * 64 + lane) * 3;
    if (!pr.inside) {
        o[0] = o[1] = o[2] = 0.0f; // clipped border pixels are written as 0
    } else {
        Rng r;
        r.base = a.mt_state + (size_t)slot * (2 * MT_N * 64) + lane;
        rng_seed(r, ((pr.px << 16u) | pr.py) ^ 0xb0ae9d99u);
        rng_store(a, p, r);
        uint32_t i = 0;
        while (i < a.spp && !start_sample(sc, a, p, pr, i, q)) ++i; // max_depth <= 0: L = 0 per sample
        a.sample[p] = i;
        if (i >= a.spp) { // no path makes a query: the pixel is sum(0) / spp
            o[0] = o[1] = o[2] = 0.0f;
            samples = a.spp;
        }
    }
    slot_count(a.wstat + (size_t)slot * ST_N, ST_SAMPLES, samples);
}

__global__ void __launch_bounds__(WP_BLOCK) wp_init(Scene sc, PathArgs a)
{
    extern __shared__ uint32_t lds[];
    const Rsq     q{ sc.rsqrt_entries, sc.rsqrt_bits, sc.rsqrt_zero, sc.rsqrt_denorm, sc.rsqrt_shift, sc.rsqrt_hi };
    const int32_t slot = (int32_t)((blockIdx.x * WP_BLOCK + threadIdx.x) >> 6);
    if (slot >= a.slots) return;
    const int32_t pos = slot < a.num_tiles ? slot : -1;
    if ((threadIdx.x & 63) == 0) a.slot_tile[slot] = pos;
    if (pos >= 0) slot_begin(sc, a, slot, pos, q);
}

// ---------------------------------------------------------------------------- trace
__global__ void __launch_bounds__(WP_BLOCK) wp_trace(Scene sc, PathArgs a)
{
    extern __shared__ uint32_t lds[];
    const int32_t slot = (int32_t)((blockIdx.x * WP_BLOCK + threadIdx.x) >> 6);
    if (slot >= a.slots || a.slot_tile[slot] < 0) return;
    const int     lane = threadIdx.x & 63;
    const int64_t p    = (int64_t)slot * 64 + lane;
    const Stack   st{ lds + (threadIdx.x >> 6) * sc.stack_words * 64, lane, sc.stack_depth };
    const uint32_t kind = a.phase[p] & 0xffu;
    uint32_t       rays = 0, shadow = 0;
    if (kind != PH_DONE) {
        const float4 q0 = F(a, F_Q0, p), q1 = F(a, F_Q1, p);
        Ray          r;
        r.o = mk(q0.x, q0.y, q0.z);
        r.d = mk(q1.x, q1.y, q1.z);
        if (kind == PH_SHADOW) { // occluded(): Scene::intersect_p (Integrator.cpp:503)
            const bool occ = scene_any(sc, r, q0.w, q1.w, st);
            F(a, F_LH, p).w = __uint_as_float(occ ? 2u : 0u);
            rays = shadow = 1;
        } else {
            // intersect_lights (+ intersect for an extension ray, Integrator.cpp:557-562;
            // + intersect_p for the MIS ray, :532-533)
            const LightHit lh  = scene_intersect_lights(sc, r, q0.w, k_infinite, st);
            uint32_t       flg = lh.hit ? 1u : 0u;
            if (lh.hit) flg |= (uint32_t)(lh.env + 1) << 2;
            rays = 1;
            if (kind == PH_EXT) {
                const Hit h   = scene_intersect(sc, r, q0.w, lh.hit ? lh.t : k_infinite, st);
                F(a, F_H, p)  = make_float4(h.t, __uint_as_float(h.code), h.beta, h.gamma);
            } else if (lh.hit) {
                if (scene_any(sc, r, q0.w, k_infinite, st)) flg |= 2u;
                ++rays;
                ++shadow;
            }
            F(a, F_LH, p) = make_float4(lh.L.r, lh.L.g, lh.L.b, __uint_as_float(flg));
        }
    }
    unsigned long long* ws = a.wstat + (size_t)slot * ST_N;
    slot_count(ws, ST_RAYS, rays);
    slot_count(ws, ST_SHADOW, shadow);
}

// ---------------------------------------------------------------------------- shade
__device__ __forceinline__ rgb lh_radiance(const Scene& sc, float4 lh, f3 dir, const Rsq& q)
{
    LightHit h;
    const uint32_t flg = __float_as_uint(lh.w);
    h.hit = (flg & 1u) != 0;
    h.L   = mkc(lh.x, lh.y, lh.z);
    h.env = (int32_t)(flg >> 2) - 1;
    return light_hit_L(sc, h, dir, q);
}

enum Act { A_EXT, A_SHADOW, A_MIS, A_NEE, A_LIGHT_DONE, A_FINAL, A_PATH_END, A_STOP };

template <int INTEG>
__device__ void shade_pixel(const Scene& sc, const PathArgs& a, int64_t p, const Pix& pr, Rng& rng, const Rsq& q,
                            bool& pixel_done)
{
    constexpr bool NEE = INTEG == SP_INTEGRATOR_ITERATIVE_RRNEE;
    constexpr bool RR  = INTEG != SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE;
    constexpr float rr_cut = 0.1f;
    const uint32_t ph   = a.phase[p];
    int            li   = (int)(ph >> 8);
    int            act  = (ph & 0xffu) == PH_EXT ? A_EXT : (ph & 0xffu) == PH_SHADOW ? A_SHADOW : A_MIS;
    float4         fl   = F(a, F_L, p);
    float4         ft   = F(a, F_T, p);
    rgb            L    = mkc(fl.x, fl.y, fl.z);
    rgb            thr  = mkc(fl.w, ft.x, ft.y);
    // bounce state (RRNEE: kept in HBM between the NEE queries)
    f3    sp = mk(0, 0, 0), sn = mk(0, 0, 0), swo = mk(0, 0, 0), sdir = mk(0, 0, 0);
    rgb   scol = mkc(0, 0, 0);
    float spdf = 0.0f;
    int   mat  = (int)__float_as_uint(ft.z);
    bool  have_bounce = false; // sp/sn/swo/sdir/scol loaded or computed in registers
    auto load_bounce = [&]() {
        if (have_bounce) return;
        const float4 a0 = F(a, F_P, p), a1 = F(a, F_N, p), a2 = F(a, F_WO, p), a3 = F(a, F_SD, p), a4 = F(a, F_SC, p);
        sp   = mk(a0.x, a0.y, a0.z);
        sn   = mk(a1.x, a1.y, a1.z);
        swo  = mk(a2.x, a2.y, a2.z);
        sdir = mk(a3.x, a3.y, a3.z);
        scol = mkc(a4.x, a4.y, a4.z);
        spdf = ft.w;
        have_bounce = true;
    };
    rgb Lr = mkc(0, 0, 0);
    while (act != A_STOP) {
        if (act == A_EXT) {
            const float4 q0 = F(a, F_Q0, p), q1 = F(a, F_Q1, p), hr = F(a, F_H, p);
            Ray          ray;
            ray.o = mk(q0.x, q0.y, q0.z);
            ray.d = mk(q1.x, q1.y, q1.z);
            Hit h;
            h.t     = hr.x;
            h.code  = __float_as_uint(hr.y);
            h.beta  = hr.z;
            h.gamma = hr.w;
            if (h.code != 0xffffffffu) {
                const Isect   is = finish_hit(sc, h, ray, q);
                const f3      wo = neg(ray.d);
                const MSample s  = material_sample(sc, is.material, wo, is.n, rng, q);
                if (s.pdf == 0.0f || cblack(s.color)) { act = A_PATH_END; continue; }
                sp = is.p; sn = is.n; swo = wo; sdir = s.dir; scol = s.color; spdf = s.pdf; mat = is.material;
                have_bounce = true;
                if constexpr (NEE) {
                    li  = 0;
                    act = A_NEE;
                } else {
                    act = A_FINAL;
                }
            } else {
                if (__float_as_uint(F(a, F_LH, p).w) & 1u) L = cadd(L, cmul(thr, lh_radiance(sc, F(a, F_LH, p), ray.d, q)));
                act = A_PATH_END;
            }
        } else if (act == A_NEE) { // estimate_direct_mis, first half (Integrator.cpp:497-505)
            if (li >= sc.n_lights) { act = A_FINAL; continue; }
            load_bounce();
            const Light   l  = sc.lights[li]; // per-lane index: vector load (uload_* needs a wave-uniform address)
            const LSample ls = light_sample(sc, l, sp, sn, next2D(rng), q);
            if (ls.pdf == 0.0f || cblack(ls.L)) { Lr = mkc(0, 0, 0); act = A_LIGHT_DONE; continue; }
            put_query(a, p, ls.ray, ls.tmin, ls.tmax);
            F(a, F_LS, p) = make_float4(ls.L.r, ls.L.g, ls.L.b, 0.0f);
            float4 fp     = make_float4(sp.x, sp.y, sp.z, ls.pdf);
            F(a, F_P, p)  = fp;
            a.phase[p]    = PH_SHADOW | ((uint32_t)li << 8);
            act           = A_STOP;
        } else if (act == A_SHADOW) { // second half: occluded -> black; eval, pdf, MIS sample
            load_bounce();
            Lr = mkc(0, 0, 0);
            if (__float_as_uint(F(a, F_LH, p).w) & 2u) { act = A_LIGHT_DONE; continue; }
            const float4 q1  = F(a, F_Q1, p);
            const f3     wi  = mk(q1.x, q1.y, q1.z);
            const float4 lsr = F(a, F_LS, p);
            const rgb    lsL = mkc(lsr.x, lsr.y, lsr.z);
            const float  lsp = F(a, F_P, p).w;
            const rgb    be  = material_eval(sc, mat, swo, wi, sn, rng, q);
            if (!cblack(be)) {
                const float bp = material_pdf(sc, mat, swo, wi, sn, rng, q);
                if (bp > 0.0f) {
                    const float w = balance(lsp, lsp + bp);
                    Lr            = cadd(Lr, cscale(cmul(be, lsL), abs_f(dot(wi, sn)) * w / lsp));
                }
            }
            const MSample ms = material_sample(sc, mat, swo, sn, rng, q);
            if (ms.pdf == 0.0f || cblack(ms.color)) { act = A_LIGHT_DONE; continue; }
            const Light l  = sc.lights[li];
            const float lp = light_pdf(sc, l, sp, ms.dir);
            if (lp == 0.0f) { act = A_LIGHT_DONE; continue; }
            const float w = balance(ms.pdf, ms.pdf + lp);
            Ray         mr;
            mr.o = sp;
            mr.d = ms.dir;
            put_query(a, p, mr, ray_offset(sn, ms.dir), k_infinite);
            F(a, F_LR, p) = make_float4(Lr.r, Lr.g, Lr.b, 0.0f);
            F(a, F_MC, p) = make_float4(ms.color.r, ms.color.g, ms.color.b, 0.0f);
            F(a, F_N, p)  = make_float4(sn.x, sn.y, sn.z, ms.pdf);
            F(a, F_WO, p) = make_float4(swo.x, swo.y, swo.z, w);
            a.phase[p]    = PH_MIS | ((uint32_t)li << 8);
            act           = A_STOP;
        } else if (act == A_MIS) { // third part: light reached along the material sample
            load_bounce();
            const float4 lr = F(a, F_LR, p);
            Lr              = mkc(lr.x, lr.y, lr.z);
            const float4 lh = F(a, F_LH, p);
            const uint32_t flg = __float_as_uint(lh.w);
            if ((flg & 1u) && !(flg & 2u)) {
                const float4 q1  = F(a, F_Q1, p);
                const f3     md  = mk(q1.x, q1.y, q1.z);
                const float4 mc  = F(a, F_MC, p);
                const float  mpd = F(a, F_N, p).w;
                const float  w   = F(a, F_WO, p).w;
                const rgb    Ll  = lh_radiance(sc, lh, md, q);
                Lr = cadd(Lr, cdivs(cscale(cscale(cmul(mkc(mc.x, mc.y, mc.z), Ll), abs_f(dot(md, sn))), w), mpd));
            }
            act = A_LIGHT_DONE;
        } else if (act == A_LIGHT_DONE) { // L += throughput * estimate_direct_mis(...) (Integrator.cpp:590)
            L = cadd(L, cmul(thr, Lr));
            ++li;
            act = A_NEE;
        } else if (act == A_FINAL) { // next direction, throughput, Russian roulette (:604-626)
            load_bounce();
            const float cosine = abs_f(dot(sdir, sn));
            thr                = cmul(thr, cdivs(cscale(scol, cosine), spdf));
            if (RR && (int)a.depth[p] >= sc.rr_depth) {
                const float lum = luminance(thr);
                if (lum < rr_cut) {
                    const float qv = std_max(0.05f, lum / rr_cut);
                    if (next1D(rng) < qv) {
                        thr = cdivs(thr, qv);
                    } else {
                        act = A_PATH_END;
                        continue;
                    }
                }
            }
            const uint32_t d = a.depth[p] + 1;
            if ((int)d >= sc.max_depth) { act = A_PATH_END; continue; }
            a.depth[p] = d;
            Ray r;
            r.o = sp;
            r.d = sdir;
            put_query(a, p, r, ray_offset(cosine), k_infinite);
            a.phase[p] = PH_EXT;
            act        = A_STOP;
        } else { // A_PATH_END: image(p) += integrate(...), next sample
            a.acc[p]           = a.acc[p] + L.r;
            a.acc[a.n + p]     = a.acc[a.n + p] + L.g;
            a.acc[2 * a.n + p] = a.acc[2 * a.n + p] + L.b;
            uint32_t i = a.sample[p] + 1;
            while (i < a.spp) {
                if (start_sample(sc, a, p, pr, i, q)) break;
                a.acc[p] = a.acc[p] + 0.0f; // a path with no query contributes L = 0
                a.acc[a.n + p] = a.acc[a.n + p] + 0.0f;
                a.acc[2 * a.n + p] = a.acc[2 * a.n + p] + 0.0f;
                ++i;
            }
            a.sample[p] = i;
            if (i >= a.spp) {
                a.phase[p] = PH_DONE;
                pixel_done = true;
            }
            return; // start_sample stored the new path's L / throughput
        }
    }
    // persist the path state the next shade invocation needs
    F(a, F_L, p) = make_float4(L.r, L.g, L.b, thr.r);
    F(a, F_T, p) = make_float4(thr.g, thr.b, __uint_as_float((uint32_t)mat), spdf);
    if constexpr (NEE) {
        if (have_bounce) {
            const float4 fp = F(a, F_P, p);
            F(a, F_P, p)  = make_float4(sp.x, sp.y, sp.z, fp.w);
            const float4 fn = F(a, F_N, p);
            F(a, F_N, p)  = make_float4(sn.x, sn.y, sn.z, fn.w);
            const float4 fw = F(a, F_WO, p);
            F(a, F_WO, p) = make_float4(swo.x, swo.y, swo.z, fw.w);
            F(a, F_SD, p) = make_float4(sdir.x, sdir.y, sdir.z, 0.0f);
            F(a, F_SC, p) = make_float4(scol.r, scol.g, scol.b, 0.0f);
        }
    }
}

template <int INTEG, int MINW>
__global__ void __launch_bounds__(WP_BLOCK, MINW) wp_shade(Scene sc, PathArgs a)
{
    extern __shared__ uint32_t lds[];
    const int rs_words = rsqrt_words(sc);
    for (int i = threadIdx.x; i < rs_words; i += WP_BLOCK) lds[i] = sc.rsqrt_entries[i];
    libm_lds_init(threadIdx.x, WP_BLOCK);
    __syncthreads();
    const int32_t slot = (int32_t)((blockIdx.x * WP_BLOCK + threadIdx.x) >> 6);
    if (slot >= a.slots) return;
    const int32_t pos = a.slot_tile[slot];
    if (pos < 0) return;
    const Rsq      q{ lds, sc.rsqrt_bits, sc.rsqrt_zero, sc.rsqrt_denorm, sc.rsqrt_shift, sc.rsqrt_hi };
    const uint32_t lane = threadIdx.x & 63u;
    const int64_t  p    = (int64_t)slot * 64 + lane;
    const Pix      pr   = pixel_of(sc, a, pos, lane);
    bool           live = (a.phase[p] & 0xffu) != PH_DONE;
    uint32_t       draws = 0, samples = 0;
    if (live) {
        Rng rng = rng_load(a, p);
        rng_prepare(rng);
        bool done = false;
        shade_pixel<INTEG>(sc, a, p, pr, rng, q, done);
        draws = rng.draws;
        rng_store(a, p, rng);
        if (done) { // image(p) /= num_pixel_samples (main.cpp:102)
            rgb s = mkc(a.acc[p], a.acc[a.n + p], a.acc[2 * a.n + p]);
            s     = cdivs(s, (float)a.spp);
            float* o = a.out + ((size_t)pos * 64 + lane) * 3;
            o[0] = s.r;
            o[1] = s.g;
            o[2] = s.b;
            samples = a.spp;
            live    = false;
        }
    }
    unsigned long long* ws = a.wstat + (size_t)slot * ST_N;
    slot_count(ws, ST_DRAWS, draws);
    slot_count(ws, ST_SAMPLES, samples);
    // all 64 pixels done: the slot takes the next tile of the caller's list
    if (__ballot(live) == 0) {
        int32_t next = 0;
        if (lane == 0) next = atomicAdd(a.next_tile, 1);
        next = __shfl(next, 0, 64);
        if (next < a.num_tiles) {
            if (lane == 0) a.slot_tile[slot] = next;
            slot_begin(sc, a, slot, next, q);
        } else {
            if (lane == 0) {
                a.slot_tile[slot] = -1;
                atomicSub(a.active, 1);
            }
        }
    }
}

__global__ void __launch_bounds__(WP_BLOCK) wp_stats(PathArgs a, unsigned long long* counters)
{
    __shared__ unsigned long long part[ST_N][WP_BLOCK / 64];
    unsigned long long v[ST_N] = {};
    for (int64_t i = (int64_t)blockIdx.x * WP_BLOCK + threadIdx.x; i < a.slots; i += (int64_t)gridDim.x * WP_BLOCK)
        for (int k = 0; k < ST_N; ++k) v[k] += a.wstat[i * ST_N + k];
    for (int k = 0; k < ST_N; ++k) {
        unsigned long long x = v[k];
        for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
        if ((threadIdx.x & 63) == 0) part[k][threadIdx.x >> 6] = x;
    }
    __syncthreads();
    if (threadIdx.x < ST_N) {
        unsigned long long x = 0;
        for (int j = 0; j < WP_BLOCK / 64; ++j) x += part[threadIdx.x][j];
        if (x) atomicAdd(counters + threadIdx.x, x); // rays, shadow, samples, draws
    }
}

using ShadeFn = void (*)(Scene, PathArgs);
ShadeFn shade_kernel(int integ)
{
    switch (integ) {
    case SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE: return wp_shade<SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE, 4>;
    case SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE_RR: return wp_shade<SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE_RR, 4>;
    case SP_INTEGRATOR_ITERATIVE_RRNEE: return wp_shade<SP_INTEGRATOR_ITERATIVE_RRNEE, 4>;
    default: return nullptr;
    }
}

} // namespace

bool wpath_supports(int integ) { return shade_kernel(integ) != nullptr; }

size_t wpath_bytes_per_slot() { return 64 * ((size_t)NF * 16 + 4 * 4 + 3 * 4 + 2 * MT_N * 8) + ST_N * 8 + 4; }

hipError_t wpath_render(const Scene& sc, const WPathRun& r, hipStream_t stream, int* iterations)
{
    PathArgs a{};
    a.slots     = r.slots;
    a.n         = (int64_t)r.slots * 64;
    a.tile_ids  = r.tile_ids;
    a.num_tiles = r.num_tiles;
    a.tiles_x   = r.tiles_x;
    a.spp       = r.spp;
    a.out       = r.out;
    // carve the state buffer (every array 256-byte aligned; n is a multiple of 64)
    char* b    = static_cast<char*>(r.buf);
    auto  take = [&](size_t bytes) { char* x = b; b += (bytes + 255) & ~(size_t)255; return x; };
    a.mt_state  = reinterpret_cast<uint64_t*>(take((size_t)a.n * 2 * MT_N * 8));
    a.ps        = reinterpret_cast<float4*>(take((size_t)NF * a.n * 16));
    a.acc       = reinterpret_cast<float*>(take((size_t)a.n * 12));
    a.phase     = reinterpret_cast<uint32_t*>(take((size_t)a.n * 4));
    a.rstate    = reinterpret_cast<uint32_t*>(take((size_t)a.n * 4));
    a.sample    = reinterpret_cast<uint32_t*>(take((size_t)a.n * 4));
    a.depth     = reinterpret_cast<uint32_t*>(take((size_t)a.n * 4));
    a.slot_tile = reinterpret_cast<int32_t*>(take((size_t)a.slots * 4));
    a.wstat     = reinterpret_cast<unsigned long long*>(take((size_t)a.slots * ST_N * 8));
    a.next_tile = r.ctl;
    a.active    = r.ctl + 1;
    ShadeFn shade = shade_kernel(r.integrator);
    if (!shade) return hipErrorInvalidValue;
    const int32_t init_ctl[2] = { (int32_t)std::min<int64_t>(r.slots, r.num_tiles), (int32_t)std::min<int64_t>(r.slots, r.num_tiles) };
    hipError_t    e           = hipMemcpyAsync(r.ctl, init_ctl, sizeof init_ctl, hipMemcpyHostToDevice, stream);
    if (e != hipSuccess) return e;
    if ((e = hipMemsetAsync(a.wstat, 0, (size_t)a.slots * ST_N * 8, stream)) != hipSuccess) return e;
    const unsigned grid      = (unsigned)((a.slots + (WP_BLOCK / 64) - 1) / (WP_BLOCK / 64));
    const size_t   stack_lds = (size_t)(WP_BLOCK / 64) * sc.stack_words * 64 * 4;
    const size_t   rs_lds    = (size_t)rsqrt_words(sc) * 4;
    hipLaunchKernelGGL(wp_init, dim3(grid), dim3(WP_BLOCK), 0, stream, sc, a);
    // (trace, shade) rounds until no slot holds a tile.  The active count is copied to host
    // memory after every WP_POLL rounds and read one batch later (no stall in the loop).
    std::vector<hipEvent_t> ev;
    int                     it = 0;
    int                     batch = 0;
    volatile int32_t*       host_active = r.host_active; // pinned, 2 entries (ping-pong)
    host_active[0] = host_active[1] = 1;
    bool                    finished = false;
    hipEvent_t              evs[2]   = { r.poll_ev[0], r.poll_ev[1] };
    while (!finished) {
        for (int k = 0; k < WP_POLL; ++k, ++it) {
            hipLaunchKernelGGL(wp_trace, dim3(grid), dim3(WP_BLOCK), stack_lds, stream, sc, a);
            hipLaunchKernelGGL(shade, dim3(grid), dim3(WP_BLOCK), rs_lds, stream, sc, a);
        }
        if ((e = hipGetLastError()) != hipSuccess) return e;
        const int slotb = batch & 1;
        if ((e = hipMemcpyAsync((void*)(host_active + slotb), a.active, 4, hipMemcpyDeviceToHost, stream)) != hipSuccess) return e;
        if ((e = hipEventRecord(evs[slotb], stream)) != hipSuccess) return e;
        if (batch > 0) { // the previous batch's count
            if ((e = hipEventSynchronize(evs[slotb ^ 1])) != hipSuccess) return e;
            if (host_active[slotb ^ 1] == 0) finished = true;
        }
        ++batch;
        // runaway guard: no slot can need more rounds than every tile's every query in sequence
        const double bound = (double)r.num_tiles * r.spp * ((double)std::max(sc.max_depth, 0) * (1 + 2 * sc.n_lights) + 1) + 4 * WP_POLL;
        if ((double)it > bound) return hipErrorUnknown;
    }
    hipLaunchKernelGGL(wp_stats, dim3(64), dim3(WP_BLOCK), 0, stream, a, r.counters);
    if (iterations) *iterations = it;
    return hipGetLastError();
}

} // namespace spd
