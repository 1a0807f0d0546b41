// sp_wave.hip -- wavefront form of DirectLightingIntegrator (Integrators/Integrator.cpp:277).
//
// The megakernel (sp_mega.hip) keeps traversal and shading in one ~190-VGPR kernel: two waves
// per SIMD, half of all wave cycles stalled on dependent BVH node loads.  Here each sample of
// every pixel in flight is split at its ray queries:
//
//   wf_init     seed each pixel's mt19937_64, zero its running sum        (main.cpp:73, 94)
//   per sample i = 0..spp-1:
//     wf_primary  R2 jitter -> camera ray -> intersect_lights + intersect  (Scene.h:69-79)
//                 traversal only: small register footprint, LDS stack, high occupancy;
//                 a light-only hit adds its radiance to the sum right here
//     wf_shade    closest hit -> shading frame -> per light: Light::sample + Material::eval
//                 (all RNG draws of the sample, in reference order); writes one shadow ray
//                 + contribution per light and appends the pixel to the shadow queue
//                 (wave ballot + one atomic per wave: active-ray compaction)
//     wf_shadow   compacted queue -> Scene::intersect_p per light, in light order ->
//                 L = sum of unoccluded contributions -> sum += L
//   wf_resolve  sum / spp -> tile-packed output                           (main.cpp:102)
//
// The floating-point sequence per pixel is exactly the megakernel's: contributions are formed
// in wf_shade with the reference's expression and summed in wf_shadow in light order, so the
// two pipelines are bit-identical (tests/test_gpu_parity.py).  Skipping the sum for pixels with
// no unoccluded light is exact too: the running sum is never -0, so sum + 0 == sum.
//
// HBM layout (n = pixels in flight = tiles * 64, pixel slot p = tile_slot * 64 + morton lane):
//   acc[3][n] f32 SoA | rstate[n] u32 {idx | cur<<16 | ready<<17} | hit[n] float4 {t, code,
//   beta, gamma} | shp[n] float4 {p.xyz, light mask} | sh[light][n][2] float4 {wi.xyz, tmin},
//   {contrib.rgb, tmax} | queue[n] u32 | mt[tile][buf][312][64] u64 (as in the megakernel).
// RNG draw-ahead window (sp_path.hpp Rng): off in the wavefront kernels, where it measured
// 1-2 % slower (it pays off in the megakernel, 2 words ahead).
#ifndef SP_WAVE_RNG_PF
#define SP_WAVE_RNG_PF 0
#endif
#define SP_RNG_PF SP_WAVE_RNG_PF
// Rows of the RNG stream wf_shade pulls into L2 ahead of a glossy hit's draws (rng_touch; 0 = off).
#ifndef SP_WAVE_RNG_TOUCH
#define SP_WAVE_RNG_TOUCH 68
#endif
#include "sp_path.hpp"
#include "sp_wave.hpp"

#include <cstdlib>

namespace spd {

constexpr int WF_BLOCK = 256;
#ifndef WF_PRIM_WAVES
#define WF_PRIM_WAVES 1 // camera-ray kernel: no occupancy request (the binary walk needs few registers)
#endif
#ifndef WF_TRAV_WAVES
#define WF_TRAV_WAVES 8 // waves per SIMD requested for wf_shadow (64 VGPRs, 20 B spill; 6 / 7 / 8 measured
                        // 2245 / 2247 / 2282 Mrays/s without SLP vectorisation, profiles/r02/s5)
#endif
constexpr int QSEG     = 32; // shadow-queue segments (one counter each, QSTRIDE words apart)
constexpr int QSTRIDE  = 32;
constexpr int QFETCH   = 16; // fetch counter of a segment: QFETCH words after its fill counter
__host__ __device__ inline size_t qseg_cap(int64_t n) { return (size_t)64 * (size_t)(((n >> 6) + QSEG - 1) / QSEG); }

struct PixelRef {
    uint32_t px, py;
    bool     inside;
};

// Internal slot -> caller's slot.  With P parts the caller's tiles are dealt in blocks of ilv
// tiles, round-robin (part k = blocks k, k + P, k + 2P, ...; a last partial block goes to the
// part whose turn it is), so every part sees a similar mix of cheap (sky) and expensive tiles
// while neighbouring tiles stay together.  Internal slots hold part 0's tiles, then part 1's, ...
__host__ __device__ inline int64_t part_slots(int64_t slots, int64_t ilv, int parts, int k)
{
    const int64_t full = slots / ilv, rem = slots % ilv;
    const int64_t nb   = (full > k) ? (full - k + parts - 1) / parts : 0;
    return nb * ilv + ((full % parts == k) ? rem : 0);
}
__device__ __forceinline__ int64_t caller_slot(const WaveArgs& w, int64_t slot)
{
    if (!w.interleave) return slot;
    const int64_t ilv = w.interleave, slots = w.n >> 6;
    int           k   = 0;
    int64_t       s   = slot;
    while (k + 1 < w.n_parts) {
        const int64_t ns = part_slots(slots, ilv, w.n_parts, k);
        if (s < ns) break;
        s -= ns;
        ++k;
    }
    return ((s / ilv) * w.n_parts + k) * ilv + s % ilv;
}

__device__ __forceinline__ PixelRef pixel_of(const Scene& sc, const WaveArgs& w, int64_t p)
{
    const int64_t  slot = caller_slot(w, p >> 6);
    const uint32_t lane = (uint32_t)p & 63u;
    const int32_t  tile = w.tile_ids ? w.tile_ids[slot] : (int32_t)slot;
    PixelRef       r;
    r.px     = (uint32_t)((tile % w.tiles_x) * 8) + morton_decode_1(lane);
    r.py     = (uint32_t)((tile / w.tiles_x) * 8) + morton_decode_1(lane >> 1);
    r.inside = r.px < (uint32_t)sc.width && r.py < (uint32_t)sc.height; // unsigned: a negative id is outside
    return r;
}

// RSequenceSampler::get_next_2D (math/Sampler.h:158) + PerspectiveCamera::generate_ray_impl
// (Cameras/Camera.h:119) -- same expression as the megakernel's sample loop.
__device__ __forceinline__ Ray camera_ray(const Scene& sc, const PixelRef& pr, uint32_t i, const Rsq& q)
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

// Statistics without same-address atomics: each wave adds its sums into its own slot of
// WaveArgs::wstat (plain read-modify-write; a slot belongs to one wave per launch); wf_stats
// reduces the slots once per frame.  32400 waves x 3 kernels x 256 samples of device-scope
// atomics on one address would serialise at the memory side.
enum { ST_RAYS = 0, ST_SHADOW = 1, ST_SAMPLES = 2, ST_DRAWS = 3, ST_HITS = 4, ST_N = 5 };
__device__ __forceinline__ void wave_count(unsigned long long* slot, int k, uint32_t v)
{
    uint32_t s = v;
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
    if ((threadIdx.x & 63) == 0 && s) slot[k] += s;
}

// Diagnostic per-wave record (only when WaveArgs::diag is set): {t0, t1 (s_memrealtime,
// 100 MHz), node steps | active lanes << 32, HW_ID | XCC_ID << 32}.
__device__ __forceinline__ void diag_record(unsigned long long* rec, uint64_t t0, uint32_t steps, uint32_t lanes)
{
    if ((threadIdx.x & 63) != 0) return;
    const uint64_t t1  = __builtin_amdgcn_s_memrealtime();
    const uint32_t hw  = __builtin_amdgcn_s_getreg((4) | (0 << 6) | ((32 - 1) << 11));
    const uint32_t xcc = __builtin_amdgcn_s_getreg((20) | (0 << 6) | ((16 - 1) << 11));
    rec[0]             = t0;
    rec[1]             = t1;
    rec[2]             = (uint64_t)steps | ((uint64_t)lanes << 32);
    rec[3]             = (uint64_t)hw | ((uint64_t)xcc << 32);
}

__device__ __forceinline__ Rng rng_load(const WaveArgs& w, int64_t p)
{
    Rng            r;
    const uint32_t st = w.rstate[p];
    r.base  = w.mt_state + (size_t)(p >> 6) * (2 * (size_t)MT_GEN_WORDS) + (size_t)(p & 63) * MT_BLK;
    r.idx   = (int)(st & 0xffffu);
    r.cur   = (int)((st >> 16) & 1u);
    r.ready = (int)((st >> 17) & 1u);
    r.draws = 0;
    return r;
}
__device__ __forceinline__ void rng_store(const WaveArgs& w, int64_t p, const Rng& r)
{
    w.rstate[p] = (uint32_t)r.idx | ((uint32_t)r.cur << 16) | ((uint32_t)r.ready << 17);
}

__global__ void __launch_bounds__(WF_BLOCK) wf_init(Scene sc, WaveArgs w)
{
    const int64_t p = w.pb + (int64_t)blockIdx.x * WF_BLOCK + threadIdx.x;
    if (p >= w.pe) return;
    const PixelRef pr = pixel_of(sc, w, p);
    w.acc[p] = 0.0f;
    w.acc[w.n + p] = 0.0f;
    w.acc[2 * w.n + p] = 0.0f;
    if (!pr.inside) {
        w.rstate[p] = 0;
        return;
    }
    Rng r;
    r.base = w.mt_state + (size_t)(p >> 6) * (2 * (size_t)MT_GEN_WORDS) + (size_t)(p & 63) * MT_BLK;
    rng_seed(r, ((pr.px << 16u) | pr.py) ^ 0xb0ae9d99u); // get_integrator_sampler (main.cpp:73)
    rng_store(w, p, r);
}

// Primary query: Integrator::integrate's intersect_lights + intersect (Integrator.cpp:277-283).
__global__ void __launch_bounds__(WF_BLOCK, WF_PRIM_WAVES) wf_primary(Scene sc, WaveArgs w, uint32_t sample)
{
    extern __shared__ uint32_t lds[];
    const int64_t p    = w.pb + (int64_t)blockIdx.x * WF_BLOCK + threadIdx.x;
    const int     lane = threadIdx.x & 63;
    if (blockIdx.x == 0 && threadIdx.x < QSEG) { // previous sample's shadow kernels are done
        w.qcount[threadIdx.x * QSTRIDE]          = 0u;
        w.qcount[threadIdx.x * QSTRIDE + QFETCH] = 0u;
    }
    if (p >= w.pe) return;
    const uint64_t t0 = w.diag ? __builtin_amdgcn_s_memrealtime() : 0;
    const PixelRef pr = pixel_of(sc, w, p);
    float4         hrec = make_float4(0.0f, __uint_as_float(0xffffffffu), 0.0f, 0.0f);
    uint32_t       rays = 0, hits = 0;
    if (pr.inside && sc.max_depth > 0) {
        const Rsq   q{ sc.rsqrt_entries };
        const Ray   ray  = camera_ray(sc, pr, sample, q);
        float       tmax = k_infinite;
        const Stack st{ lds + (threadIdx.x >> 6) * sc.stack_words * 64, lane, sc.stack_depth };
        const LightHit lh = scene_intersect_lights(sc, ray, k_ray_epsilon, tmax, st);
        if (lh.hit) tmax = lh.t;
        const Hit h = scene_intersect(sc, ray, k_ray_epsilon, tmax, st);
        rays        = 1;
        if (h.code != 0xffffffffu) {
            hrec = make_float4(h.t, __uint_as_float(h.code), h.beta, h.gamma);
            hits = 1;
        } else if (lh.hit) {
            const rgb L = cadd(mkc(0, 0, 0), cmul(mkc(1, 1, 1), light_hit_L(sc, lh, ray.d, q)));
            w.acc[p]           = w.acc[p] + L.r;
            w.acc[w.n + p]     = w.acc[w.n + p] + L.g;
            w.acc[2 * w.n + p] = w.acc[2 * w.n + p] + L.b;
        }
    }
    w.hit[p] = hrec;
    if (w.diag) diag_record(w.diag + (size_t)(p >> 6) * 4, t0, 0, (uint32_t)__popcll(__ballot(pr.inside)));
    unsigned long long* slot = w.wstat + (size_t)(p >> 6) * ST_N;
    wave_count(slot, ST_RAYS, rays);
    wave_count(slot, ST_HITS, hits);
}

// Shading: direct_nee's sampling half (Integrator.cpp:287-296).
template <int MINW>
__global__ void __launch_bounds__(WF_BLOCK, MINW) wf_shade(Scene sc, WaveArgs w, uint32_t sample)
{
    extern __shared__ uint32_t lds[];
#if SP_WAVE_RNG_TOUCH
    __shared__ uint32_t rng_sink_words[64]; // LDS-DMA target of rng_touch, never read
    auto* rng_sink = (__attribute__((address_space(3))) void*)rng_sink_words;
#endif
    const int rs_words = rsqrt_words(sc);
    for (int i = threadIdx.x; i < rs_words; i += WF_BLOCK) lds[i] = sc.rsqrt_entries[i];
    libm_lds_init(threadIdx.x, WF_BLOCK);
    __syncthreads();
    const int64_t p = w.pb + (int64_t)blockIdx.x * WF_BLOCK + threadIdx.x;
    if (p >= w.pe) return;
    const PixelRef pr = pixel_of(sc, w, p);
    uint32_t       mask = 0, draws = 0;
#ifdef SP_SHADE_PROF
    // per-wave timeline of the stages (SP_WAVE_DIAG with a -DSP_SHADE_PROF build): the latest
    // time any lane reached each point (s_memrealtime, 100 MHz)
    uint64_t tp[6] = { __builtin_amdgcn_s_memrealtime(), 0, 0, 0, 0, 0 };
#define SP_STAMP(k) (tp[k] = __builtin_amdgcn_s_memrealtime())
#else
#define SP_STAMP(k) ((void)0)
#endif
    if (pr.inside) {
        const Rsq q{ lds };
        Rng       rng = rng_load(w, p);
        rng_prepare(rng);
        SP_STAMP(1);
        const float4 hrec = w.hit[p];
        Hit          h;
        h.t     = hrec.x;
        h.code  = __float_as_uint(hrec.y);
        h.beta  = hrec.z;
        h.gamma = hrec.w;
        if (h.code != 0xffffffffu) {
            const Ray   ray = camera_ray(sc, pr, sample, q);
            const Isect is  = finish_hit(sc, h, ray, q);
            const f3    wo  = neg(ray.d);
#if SP_WAVE_RNG_TOUCH
            // a glossy hit draws 2 + 32 words per light (light sample, 16-sample rho estimate)
            if (material_has_rho(sc, is.material)) rng_touch(rng, std::min(34 * sc.n_lights, SP_WAVE_RNG_TOUCH), rng_sink);
#endif
            SP_STAMP(2);
            for (int li = 0; li < sc.n_lights; ++li) {
                const Light   l  = uload_light(sc.lights + li);
                const LSample ls = light_sample(sc, l, is.p, is.n, next2D(rng), q);
                SP_STAMP(3);
                if (ls.pdf == 0.0f || cblack(ls.L)) continue;
                const f3  wi = ls.ray.d;
                const rgb f  = material_eval(sc, is.material, wo, wi, is.n, rng, q);
                SP_STAMP(4);
                if (cblack(f)) continue;
                const rgb c = cdivs(cscale(cmul(f, ls.L), abs_f(dot(wi, is.n))), ls.pdf);
                float4*   e = w.sh + ((size_t)li * w.n + p) * 2;
                e[0]        = make_float4(wi.x, wi.y, wi.z, ls.tmin);
                e[1]        = make_float4(c.r, c.g, c.b, ls.tmax);
                mask |= 1u << li;
            }
            w.shp[p] = make_float4(is.p.x, is.p.y, is.p.z, __uint_as_float(mask));
        }
        draws = rng.draws;
        rng_store(w, p, rng);
    }
#ifdef SP_SHADE_PROF
    SP_STAMP(5);
    if (w.diag) {
        for (int k = 1; k < 6; ++k) {
            uint64_t v = tp[k];
            for (int off = 32; off > 0; off >>= 1) v = max(v, (uint64_t)__shfl_xor((unsigned long long)v, off, 64));
            tp[k] = v;
        }
        if ((threadIdx.x & 63) == 0) {
            unsigned long long* r = w.diag + (size_t)(p >> 6) * 8;
            for (int k = 0; k < 6; ++k) r[k] = tp[k];
        }
    }
#endif
#undef SP_STAMP
    // Active-ray compaction: every (pixel, light) shadow ray becomes one queue item
    // (p << 5 | light).  Wave prefix sum of the per-lane counts, one atomic per wave on one of
    // QSEG segment counters (tile slot % QSEG) so that no single address serialises the chip.
    const int      lane = threadIdx.x & 63;
    const uint32_t mine = (uint32_t)__popc(mask);
    uint32_t       incl = mine;
    for (int off = 1; off < 64; off <<= 1) {
        const uint32_t v = __shfl_up(incl, off, 64);
        if (lane >= off) incl += v;
    }
    const uint32_t total = __shfl(incl, 63, 64);
    if (total) {
        const uint32_t seg  = (uint32_t)(p >> 6) % QSEG;
        uint32_t       base = 0;
        if (lane == 0) base = atomicAdd(w.qcount + seg * QSTRIDE, total);
        base            = __shfl(base, 0, 64);
        uint32_t* out   = w.queue + (size_t)seg * w.qcap + base + (incl - mine);
        uint32_t  k     = 0;
        for (uint32_t m = mask; m; m &= m - 1) out[k++] = ((uint32_t)p << 5) | (uint32_t)(__ffs(m) - 1);
    }
    wave_count(w.wstat + (size_t)(p >> 6) * ST_N, ST_DRAWS, draws);
}

// Shadow queries, one queued ray per lane: direct_nee's occlusion test (Integrator.cpp:297) ->
// vis[light][pixel].  (Persistent lanes that refill from the queue as their ray ends measured 2x
// slower: refilled lanes sit at different depths of the tree and their node fetches stop
// coalescing -- DESIGN.md §4.)
__global__ void __launch_bounds__(WF_BLOCK, WF_TRAV_WAVES) wf_shadow(Scene sc, WaveArgs w)
{
    extern __shared__ uint32_t lds[];
    const int      lane  = threadIdx.x & 63;
    const Stack    st{ lds + (threadIdx.x >> 6) * sc.any_stack_words * 64, lane, sc.any_stack_words };
    // Segment j holds the shadow pixels of tile slots j, j + QSEG, ... in arrival order.  Virtual
    // chunk v = 64 entries of segment v % QSEG starting at (v / QSEG) * 64: walking v in order
    // visits the tiles roughly in image order, which keeps neighbouring waves' BVH nodes in cache.
    const uint32_t segn   = lane < QSEG ? w.qcount[lane * QSTRIDE] : 0u;
    uint32_t       maxn   = segn;
    for (int off = 32; off > 0; off >>= 1) maxn = max(maxn, (uint32_t)__shfl_xor(maxn, off, 64));
    const uint32_t n_virt = QSEG * ((maxn + 63) / 64);
    const size_t   cap    = w.qcap;
    uint32_t       shadow = 0;
    const uint64_t t0     = w.diag ? __builtin_amdgcn_s_memrealtime() : 0;
    const uint32_t wave_g = (blockIdx.x * WF_BLOCK + threadIdx.x) >> 6;
    for (uint32_t v = wave_g; v < n_virt; v += gridDim.x * (WF_BLOCK / 64)) {
        const uint32_t j    = v % QSEG;
        const uint32_t k    = (v / QSEG) * 64 + (uint32_t)lane;
        const bool     live = k < (uint32_t)__shfl(segn, (int)j, 64);
        const uint32_t item = live ? w.queue[(size_t)j * cap + k] : 0u;
        const int64_t  p    = item >> 5;
        const uint32_t li   = item & 31u;
        float4         o    = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        float4         d = make_float4(0.0f, 0.0f, 1.0f, 0.0f), c = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (live) {
            o               = w.shp[p];
            const float4* e = w.sh + ((size_t)li * w.n + p) * 2;
            d               = e[0];
            c               = e[1];
        }
        Ray r;
        r.o = mk(o.x, o.y, o.z);
        r.d = mk(d.x, d.y, d.z);
        const bool occ = live ? scene_any(sc, r, d.w, c.w, st) : true;
        if (live) {
            ++shadow;
            w.vis[(size_t)li * w.n + p] = occ ? 0 : 1;
        }
    }
    if (w.diag)
        diag_record(w.diag + ((size_t)(w.n >> 6) + (w.pb >> 6) + (blockIdx.x * WF_BLOCK + threadIdx.x) / 64) * 4, t0, 0,
                    (uint32_t)__popcll(__ballot(shadow != 0)));
    unsigned long long* slot = w.wstat + ((size_t)w.sh_slot0 + (blockIdx.x * WF_BLOCK + threadIdx.x) / 64) * ST_N;
    wave_count(slot, ST_RAYS, shadow); // occluded() counts the query as a ray too
    wave_count(slot, ST_SHADOW, shadow);
}

// direct_nee's sum (Integrator.cpp:300): L = unoccluded contributions in light order; sum += L.
__global__ void __launch_bounds__(WF_BLOCK) wf_accum(Scene sc, WaveArgs w)
{
    const int64_t p = w.pb + (int64_t)blockIdx.x * WF_BLOCK + threadIdx.x;
    if (p >= w.pe) return;
    if (__float_as_uint(w.hit[p].y) == 0xffffffffu) return; // no geometry hit this sample
    const uint32_t mask = __float_as_uint(w.shp[p].w);
    if (!mask) return;
    rgb L = mkc(0, 0, 0);
    for (uint32_t m = mask; m; m &= m - 1) {
        const int li = __ffs(m) - 1;
        if (w.vis[(size_t)li * w.n + p]) {
            const float4 c = w.sh[((size_t)li * w.n + p) * 2 + 1];
            L              = cadd(L, mkc(c.x, c.y, c.z));
        }
    }
    w.acc[p]           = w.acc[p] + L.r;
    w.acc[w.n + p]     = w.acc[w.n + p] + L.g;
    w.acc[2 * w.n + p] = w.acc[2 * w.n + p] + L.b;
}

__global__ void __launch_bounds__(WF_BLOCK) wf_resolve(Scene sc, WaveArgs w, float* out)
{
    const int64_t p = w.pb + (int64_t)blockIdx.x * WF_BLOCK + threadIdx.x;
    if (p >= w.pe) return;
    const PixelRef pr = pixel_of(sc, w, p);
    rgb            a  = mkc(w.acc[p], w.acc[w.n + p], w.acc[2 * w.n + p]);
    if (pr.inside) a = cdivs(a, (float)w.spp); // image(p) /= num_pixel_samples (main.cpp:102)
    float* o = out + ((size_t)caller_slot(w, p >> 6) * 64 + (size_t)(p & 63)) * 3;
    o[0]     = a.r;
    o[1]     = a.g;
    o[2]     = a.b;
    wave_count(w.wstat + (size_t)(p >> 6) * ST_N, ST_SAMPLES, pr.inside ? w.spp : 0u);
}

// Frame statistics: sum the per-wave slots (a few hundred atomics per frame).
__global__ void __launch_bounds__(WF_BLOCK) wf_stats(WaveArgs w, int64_t n_slots)
{
    __shared__ unsigned long long part[ST_N][WF_BLOCK / 64];
    unsigned long long v[ST_N] = {};
    for (int64_t i = (int64_t)blockIdx.x * WF_BLOCK + threadIdx.x; i < n_slots; i += (int64_t)gridDim.x * WF_BLOCK)
        for (int k = 0; k < ST_N; ++k) v[k] += w.wstat[i * ST_N + k];
    for (int k = 0; k < ST_N; ++k) {
        unsigned long long x = v[k];
        for (int off = 32; off > 0; off >>= 1) x += __shfl_down(x, off, 64);
        if ((threadIdx.x & 63) == 0) part[k][threadIdx.x >> 6] = x;
    }
    __syncthreads();
    if (threadIdx.x < ST_N) {
        unsigned long long x = 0;
        for (int j = 0; j < WF_BLOCK / 64; ++j) x += part[threadIdx.x][j];
        const int map[ST_N] = { 0, 1, 2, 3, 4 }; // counters: rays, shadow, samples, draws, hits
        if (x) atomicAdd(w.counters + map[threadIdx.x], x);
    }
}

// ---------------------------------------------------------------------------- host side
// wf_shadow's LDS: per-wave any-hit stacks (wide-BVH depth, not the binary closest-hit depth)
static size_t wave_shadow_lds(const Scene& sc) { return (size_t)(WF_BLOCK / 64) * sc.any_stack_words * 64 * 4; }
// shading kernel occupancy: 4 / 5 / 6 waves per SIMD measured 2280 / 2306 / 2236 Mrays/s (profiles/r02/s5)
static int shade_waves_env() { return 5; }
// tiles per interleave block of the two parts: one 1080p tile row (profiles/r01 sweep: 1..16200 within 3 %)
static int32_t interleave_block_env() { return 240; }
static uint32_t diag_sample_env()
{
    const char* v = std::getenv("SP_WAVE_DIAG_SAMPLE");
    return v ? (uint32_t)std::atoi(v) : 0u;
}

size_t wave_bytes_per_pixel(int n_lights)
{
    return 3 * 4 + 4 + 16 + 16 + (size_t)n_lights * 32 + 4 + 2 * (size_t)(MT_GEN_WORDS / 64) * 8;
}
// primary/shade/resolve slots (one per tile) + persistent shadow-wave slots (at most as many)
// tile slots + persistent shadow-wave slots of both parts (each part's grid is at most
// ceil(part pixels / WF_BLOCK) blocks of WF_BLOCK / 64 waves)
size_t wave_stat_bytes(int64_t n) { return (size_t)(2 * (size_t)(n >> 6) + 8 * WF_MAX_PARTS) * ST_N * 8; }
// room for up to WF_MAX_PARTS parts (wave_render), each QSEG segments + QSEG counters
size_t wave_queue_bytes(int64_t n, int n_lights)
{
    const size_t L = (size_t)std::max(1, n_lights);
    return (QSEG * (qseg_cap(n) + (size_t)WF_MAX_PARTS * 64) * L + (size_t)WF_MAX_PARTS * QSEG * QSTRIDE) * 4 + 4096;
}

hipError_t wave_render(const Scene& sc, const WaveArgs& w, float* out, int traverse_blocks_per_cu, int n_cu,
                       hipStream_t stream, hipEvent_t* ev, const hipStream_t* aux, int n_aux, hipEvent_t fork,
                       const hipEvent_t* join, hipEvent_t* shade_done, int* parts_out)
{
    int  e    = 0;
    auto mark = [&]() {
        if (ev) (void)hipEventRecord(ev[e++], stream);
    };
    const size_t stack_lds  = (size_t)(WF_BLOCK / 64) * sc.stack_words * 64 * 4;
    const size_t shadow_lds = wave_shadow_lds(sc);
    const size_t rs_lds     = (size_t)rsqrt_words(sc) * 4;
    const unsigned grid_all = (unsigned)((w.n + WF_BLOCK - 1) / WF_BLOCK);

    // Parts: tile sets with their own queues, each driven by its own stream, so that one part's
    // traversal kernels (memory-latency bound) overlap another part's shading on the same CUs.
    // At least 256 tiles per part; SP_WAVE_PARTS (via n_aux + 1) sets the number.
    int parts = 1 + std::max(0, n_aux);
    while (parts > 1 && w.n < (int64_t)parts * 64 * 256) --parts;
    parts = std::min(parts, WF_MAX_PARTS);
    if (parts_out) *parts_out = parts;
    WaveArgs    pw[WF_MAX_PARTS];
    hipStream_t ps[WF_MAX_PARTS] = { stream, nullptr, nullptr, nullptr };
    for (int k = 1; k < parts; ++k) ps[k] = aux[k - 1];
    WaveArgs    wa    = w;
    wa.interleave     = parts > 1 ? interleave_block_env() : 0;
    wa.n_parts        = parts;
    const int64_t slots = w.n >> 6;
    int64_t       s0    = 0;
    uint32_t*     q     = w.queue;
    for (int k = 0; k < parts; ++k) {
        const int64_t ns = parts > 1 ? part_slots(slots, wa.interleave, parts, k) : slots;
        pw[k]            = wa;
        pw[k].pb         = s0 * 64;
        pw[k].pe         = (s0 + ns) * 64;
        pw[k].qcap       = qseg_cap(ns * 64) * (size_t)std::max(1, sc.n_lights); // one item per (pixel, light)
        pw[k].queue      = q;
        pw[k].qcount     = q + QSEG * pw[k].qcap;
        q += QSEG * pw[k].qcap + QSEG * QSTRIDE;
        s0 += ns;
    }
    mark();
    (void)hipMemsetAsync(w.wstat, 0, wave_stat_bytes(w.n), stream);
    hipLaunchKernelGGL(wf_init, dim3(grid_all), dim3(WF_BLOCK), 0, stream, sc, wa);
    mark();
    if (parts > 1) {
        (void)hipEventRecord(fork, stream);
        for (int k = 1; k < parts; ++k) (void)hipStreamWaitEvent(ps[k], fork, 0);
    }
    const uint32_t diag_sample = diag_sample_env();
    // waves per SIMD requested for the shading kernel (register budget vs spills)
    void (*shade)(Scene, WaveArgs, uint32_t) = wf_shade<5>;
    switch (shade_waves_env()) {
    case 3: shade = wf_shade<3>; break;
    case 4: shade = wf_shade<4>; break;
    case 6: shade = wf_shade<6>; break;
    default: break;
    }
    unsigned       grid[WF_MAX_PARTS], sgrid[WF_MAX_PARTS];
    WaveArgs       pd[WF_MAX_PARTS];
    int64_t        sh_slot = w.n >> 6;
    for (int k = 0; k < parts; ++k) {
        grid[k]  = (unsigned)((pw[k].pe - pw[k].pb + WF_BLOCK - 1) / WF_BLOCK);
        // the shadow queue never exceeds the part: a persistent grid sized to fill the chip
        sgrid[k] = (unsigned)std::max<int64_t>(1, std::min<int64_t>(grid[k], (int64_t)n_cu * traverse_blocks_per_cu));
        // statistics slots of this part's persistent shadow waves, after the tile slots
        pw[k].sh_slot0 = sh_slot;
        sh_slot += (int64_t)sgrid[k] * (WF_BLOCK / 64);
        pd[k]      = pw[k]; // diagnostics: only the launches of sample diag_sample record
        pd[k].diag = nullptr;
    }
    // With several parts the shading kernels take turns (part 0's shade, then part 1's, ...,
    // then part 0's again) through cross-stream events, so each part's traversal kernels run
    // beside another part's shading instead of all parts shading at once.
    for (uint32_t i = 0; i < w.spp; ++i) {
        for (int k = 0; k < parts; ++k) {
#ifdef SP_SHADE_PROF // the diag buffer holds the shade timeline only
            const WaveArgs& wi = pd[k];
            const WaveArgs& ws = (pw[k].diag && i == diag_sample) ? pw[k] : pd[k];
#else
            const WaveArgs& wi = (pw[k].diag && i == diag_sample) ? pw[k] : pd[k];
#endif
            hipStream_t     st = ps[k];
            hipLaunchKernelGGL(wf_primary, dim3(grid[k]), dim3(WF_BLOCK), stack_lds, st, sc, wi, i);
            if (k == 0) mark();
            if (parts > 1 && (k > 0 || i > 0)) (void)hipStreamWaitEvent(st, shade_done[(k + parts - 1) % parts], 0);
#ifdef SP_SHADE_PROF
            hipLaunchKernelGGL(shade, dim3(grid[k]), dim3(WF_BLOCK), rs_lds, st, sc, ws, i);
#else
            hipLaunchKernelGGL(shade, dim3(grid[k]), dim3(WF_BLOCK), rs_lds, st, sc, pd[k], i);
#endif
            if (parts > 1) (void)hipEventRecord(shade_done[k], st);
            if (k == 0) mark();
            hipLaunchKernelGGL(wf_shadow, dim3(sgrid[k]), dim3(WF_BLOCK), shadow_lds, st, sc, wi);
            hipLaunchKernelGGL(wf_accum, dim3(grid[k]), dim3(WF_BLOCK), 0, st, sc, wi);
            if (k == 0) mark();
        }
    }
    for (int k = 1; k < parts; ++k) {
        (void)hipEventRecord(join[k - 1], ps[k]);
        (void)hipStreamWaitEvent(stream, join[k - 1], 0);
    }
    hipLaunchKernelGGL(wf_resolve, dim3(grid_all), dim3(WF_BLOCK), 0, stream, sc, wa, out);
    const int64_t n_slots = 2 * slots + 8 * WF_MAX_PARTS;
    hipLaunchKernelGGL(wf_stats, dim3(64), dim3(WF_BLOCK), 0, stream, w, n_slots);
    mark();
    return hipGetLastError();
}

int wave_traverse_blocks_per_cu(const Scene& sc)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, wf_shadow, WF_BLOCK, wave_shadow_lds(sc)) != hipSuccess) return 1;
    return n > 0 ? n : 1;
}

} // namespace spd
