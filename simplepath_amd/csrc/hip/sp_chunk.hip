// sp_chunk.hip -- DirectLighting with each pixel's samples split into chunks that run in parallel.
//
// Why: a pixel's 256 samples draw from one std::mt19937_64 stream (main.cpp:73) in order, and
// how many words a sample draws depends on what it hit, so the megakernel runs every pixel as one
// serial chain.  On a 2-8 GPU shard of a 1080p frame the frame then ends with the slowest
// tile's chain (140 ms of a 141 ms span at 8 GPUs).  This pipeline cuts the chain
// without changing a single bit of the result:
//
//   ck_camera  every (pixel, sample) at once: R2 jitter -> camera ray -> intersect_lights +
//              intersect (Integrator.cpp:277-283).  Stores the hit record; a light-only hit or a
//              miss already has its final radiance, stored as the sample's L.
//   ck_count   per pixel, in sample order: seed the stream and advance it by each sample's draw
//              count (from ck_camera; with an image light, by replaying Light::sample, whose
//              usability then depends on the drawn numbers), writing every generation of the
//              stream into the pixel's store and the position at every chunk start.
//   ck_shade   every (tile, chunk) at once: start at the chunk's position in the store (no
//              twisting: the generations are there), run the reference's direct_nee for the
//              chunk's samples (same code as the megakernel), store each L.
//   ck_sum     per pixel: image(p) = (((0 + L_0) + L_1) + ...) / spp, in sample order.
//
// Every sample sees the same stream words and the same floating-point sequence as in the
// megakernel, and the sum runs in the same order, so the image is bit-identical
// (tests/test_gpu_parity.py).  Camera rays are traced once, and each generation of a stream is
// twisted once.  HBM per pixel-sample: 16 B hit record + 2 B draw count + 12 B radiance written
// and read back; per pixel: 2.5 KB per 312 draws of generator store.
// ck_shade reads a generator store that ck_count wrote long before, so every draw is an HBM read.
// As in the DirectLighting megakernel, the glossy estimate's 32 words are touched in advance
// (SP_RHO_TOUCH, LDS-DMA into a sink) and no draw-ahead window holds registers: 8-way shard
// 2359-2368 -> 2428-2456 Mrays/s, 2-way 2555 -> 2659, against a window of 2 without the touch
// (profiles/r02/s6/ab_chunk_touch.txt).
#ifndef SP_CHUNK_RNG_PF
#define SP_CHUNK_RNG_PF 0
#endif
#define SP_RNG_PF SP_CHUNK_RNG_PF
#define SP_RHO_TOUCH 1
// The generator store is written generation after generation by ck_count's twists and read by
// ck_shade at each chunk's position: word-interleaved rows measured best here (8-way shard 2785-2790
// Mrays/s per GPU against 2745-2765 with 4-word lane blocks; profiles/r04/rng_layout).
#ifndef SP_CHUNK_MT_BLK
#define SP_CHUNK_MT_BLK 1
#endif
#undef SP_MT_BLK
#define SP_MT_BLK SP_CHUNK_MT_BLK
#include "sp_chunk.hpp"

#include <algorithm>
#include <cstdlib>
#include "sp_mega.hpp"

namespace spd {

namespace {

constexpr uint32_t NO_HIT = 0xffffffffu;

struct Lds {
    Rsq   q;
    Stack st;
};

// shared prologue: rsqrt table + libm tables into LDS, then the wave's traversal stack
__device__ __forceinline__ Lds lds_setup(const Scene& sc, uint32_t* lds, bool stack)
{
    const int tid      = threadIdx.x;
    const int rs_words = rsqrt_words(sc);
    for (int i = tid; i < rs_words; i += 64 * WAVES_PER_BLOCK) lds[i] = sc.rsqrt_entries[i];
    libm_lds_init(tid, 64 * WAVES_PER_BLOCK);
    __syncthreads();
    Lds l{ Rsq{ lds },
           Stack{ lds + rs_words + (stack ? (tid >> 6) * sc.stack_words * 64 : 0), tid & 63, sc.stack_depth } };
    return l;
}

struct Px {
    uint32_t x, y;
    bool     inside;
};
__device__ __forceinline__ Px pixel(const Scene& sc, const ChunkArgs& a, int64_t slot, uint32_t lane)
{
    const int64_t s    = a.slot_map ? (int64_t)a.slot_map[slot] : slot;
    const int32_t tile = a.tile_ids ? a.tile_ids[s] : (int32_t)s;
    Px            p;
    p.x      = (uint32_t)((tile % a.tiles_x) * 8) + morton_decode_1(lane);
    p.y      = (uint32_t)((tile / a.tiles_x) * 8) + morton_decode_1(lane >> 1);
    p.inside = p.x < (uint32_t)sc.width && p.y < (uint32_t)sc.height; // unsigned: a negative id is outside
    return p;
}

// RSequenceSampler::get_next_2D (math/Sampler.h:158) + PerspectiveCamera::generate_ray_impl
// (Cameras/Camera.h:119), as in the megakernel's sample loop
__device__ __forceinline__ Ray camera_ray_px(const Scene& sc, const Px& p, uint32_t i, const Rsq& q)
{
    const uint32_t seed2d = ((p.x << 16u) | p.y) ^ 0x6184faf4u;
    const float    sx     = rseq_component(seed2d, sc.alpha2_0, i);
    const float    sy     = rseq_component(seed2d, sc.alpha2_1, i);
    const float    fx     = (float)(int)p.x + sx;
    const float    fy     = (float)(int)p.y + sy;
    Ray            ray;
    ray.o = sc.camera.p;
    ray.d = normalize(add(add(scale(fx, sc.camera.vx), scale(fy, sc.camera.vy)), sc.camera.vz), q);
    return ray;
}

__device__ __forceinline__ void wave_add(unsigned long long* ctr, uint64_t v)
{
    for (int off = 32; off > 0; off >>= 1) v += __shfl_down(v, off, 64);
    if ((threadIdx.x & 63) == 0 && v) atomicAdd(ctr, (unsigned long long)v);
}

__device__ __forceinline__ int64_t grab(int32_t* counter)
{
    int g = 0;
    if ((threadIdx.x & 63) == 0) g = atomicAdd(counter, 1);
    return __shfl(g, 0, 64);
}

} // namespace

// ---------------------------------------------------------------------------- camera rays
// Persistent: each wave takes items (tile, sample) w, w + W, w + 2W, ... (W = the grid's waves), so
// the LDS tables are loaded once per block instead of once per 64 camera rays (one block per item
// group used to load the RSQRTSS table and libm tables for 4 x 64 rays).
__device__ __forceinline__ void camera_item(const Scene& sc, const ChunkArgs& a, const Lds& l, uint32_t lane, int64_t item)
{
    const int64_t  slot = item % a.num_tiles;
    const uint32_t i    = (uint32_t)(item / a.num_tiles);
    const Px       px   = pixel(sc, a, slot, lane);
    const size_t   p    = (size_t)slot * 64 + lane;
    float4         rec  = make_float4(0.0f, __uint_as_float(NO_HIT), 0.0f, 0.0f);
    rgb            L    = mkc(0, 0, 0);
    uint32_t       ndraw = 0;
    if (px.inside && sc.max_depth > 0) {
        // Integrator::integrate's query (Integrator.cpp:277-283), as trace() in sp_path.hpp
        const Ray      ray = camera_ray_px(sc, px, i, l.q);
        const LightHit lh  = scene_intersect_lights(sc, ray, k_ray_epsilon, k_infinite, l.st);
        const Hit      h   = scene_intersect(sc, ray, k_ray_epsilon, lh.hit ? lh.t : k_infinite, l.st);
        if (h.code != NO_HIT) {
            rec = make_float4(h.t, __uint_as_float(h.code), h.beta, h.gamma);
            if (a.draws) ndraw = sample_draws(sc, finish_hit(sc, h, ray, l.q), neg(ray.d), l.q);
        } else if (lh.hit) {
            L = cadd(L, cmul(mkc(1, 1, 1), light_hit_L(sc, lh, ray.d, l.q)));
        }
    }
    if (a.draws) a.draws[(size_t)i * a.n_px + p] = (uint16_t)ndraw;
    a.hits[(size_t)i * a.n_px + p]               = rec;
    a.L[((size_t)i * 3 + 0) * a.n_px + p] = L.r;
    a.L[((size_t)i * 3 + 1) * a.n_px + p] = L.g;
    a.L[((size_t)i * 3 + 2) * a.n_px + p] = L.b;
}
__global__ void __launch_bounds__(64 * WAVES_PER_BLOCK) ck_camera(Scene sc, ChunkArgs a)
{
    extern __shared__ uint32_t lds[];
    const Lds      l     = lds_setup(sc, lds, true);
    const uint32_t lane  = threadIdx.x & 63u;
    const int64_t  total = a.num_tiles * (int64_t)a.spp;
    const int64_t  W     = (int64_t)gridDim.x * WAVES_PER_BLOCK;
    for (int64_t item = (int64_t)blockIdx.x * WAVES_PER_BLOCK + (threadIdx.x >> 6); item < total; item += W)
        camera_item(sc, a, l, lane, item);
}

// ------------------------------------------------------------------- stream positions (replay)
// One wave per tile (the replay is a serial chain per pixel: more waves, shorter frame).
__global__ void __launch_bounds__(64 * WAVES_PER_BLOCK) ck_count(Scene sc, ChunkArgs a)
{
    extern __shared__ uint32_t lds[];
    const Lds      l     = lds_setup(sc, lds, false);
    const uint32_t lane  = threadIdx.x & 63u;
    Rng            rng;
    rng.lin = 1; // successive generations side by side in the pixel's store
    while (true) {
        const int64_t slot = grab(a.counter);
        if (slot >= a.num_tiles) break;
        const Px     px = pixel(sc, a, slot, lane);
        const size_t p  = (size_t)slot * 64 + lane;
        rng.base        = a.gens + (size_t)slot * a.gens_per_px * MT_GEN_WORDS + (size_t)lane * MT_BLK;
        // main.cpp:73; generation 0 (the seeded state) is never drawn from, so it is not stored:
        // the seed writes generation 1 (rng_seed_twisted), the replay twists on from there
        if (px.inside) rng_seed_twisted(rng, ((px.x << 16u) | px.y) ^ 0xb0ae9d99u);
        if (a.draws) {
            // Counts known from the camera pass: the stream position before sample i is the sum
            // of the earlier counts, so the counts are summed in batches of loads that are all in
            // flight together (not one dependent load per sample), and the generations are twisted
            // after, one after the other -- the same positions (in the lazy-switch form rng_skip
            // leaves: T > 0 draws -> generation ceil(T / 312), word T - 312 (generation - 1)) and
            // the same generations as skipping sample by sample.
            const uint16_t* dp = a.draws + p;
            uint32_t        T  = 0;
            for (uint32_t i0 = 0; i0 < a.spp; i0 += 8) {
                uint32_t d[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) d[j] = (px.inside && i0 + j < a.spp) ? (uint32_t)dp[(size_t)(i0 + j) * a.n_px] : 0u;
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const uint32_t i = i0 + (uint32_t)j;
                    if (i < a.spp && i % a.chunk_len == 0) {
                        const uint32_t g = T ? (T - 1) / MT_N + 1 : 0u;
                        const uint32_t w = T ? T - (g - 1) * MT_N : (uint32_t)MT_N;
                        a.snap_ctl[(size_t)(i / a.chunk_len) * a.n_px + p] = w | (g << 16);
                    }
                    T += d[j];
                }
            }
            if (px.inside) {
                const uint32_t G = T ? (T - 1) / MT_N + 1 : 0u;
#pragma unroll 1
                for (uint32_t g = 1; g < G; ++g) mt_twist_blocked<SP_TWIST_SKIP_BLOCK>(mt_buf(rng, (int)g), mt_buf(rng, (int)g + 1));
            }
            continue;
        }
        // hit records do not depend on the stream: load sample i + 1's while sample i is replayed
        float4 next = px.inside ? a.hits[p] : make_float4(0.0f, __uint_as_float(NO_HIT), 0.0f, 0.0f);
        for (uint32_t i = 0; i < a.spp; ++i) {
            const float4 rec = next;
            if (px.inside && i + 1 < a.spp) next = a.hits[(size_t)(i + 1) * a.n_px + p];
            if (i % a.chunk_len == 0) // stream position at the start of chunk i / chunk_len
                a.snap_ctl[(size_t)(i / a.chunk_len) * a.n_px + p] = (uint32_t)rng.idx | ((uint32_t)rng.cur << 16);
            if (!px.inside) continue;
            rng_prepare(rng);
            const uint32_t code = __float_as_uint(rec.y);
            if (code == NO_HIT) continue;
            // direct_nee (sp_path.hpp): per light, 2 draws for Light::sample; if the sample is
            // usable, Material::eval draws 32 words for a glossy base (16 two-word Beckmann
            // samples of the rho estimate) unless wo.y == 0 in the shading frame, else none
            const Ray   ray = camera_ray_px(sc, px, i, l.q);
            const Hit   h{ rec.x, code, rec.z, rec.w };
            const Isect is  = finish_hit(sc, h, ray, l.q);
            const f3    wo  = neg(ray.d);
            for (int li = 0; li < sc.n_lights; ++li) {
                const Light   lt = uload_light(sc.lights + li);
                const LSample ls = light_sample(sc, lt, is.p, is.n, next2D(rng), l.q);
                if (ls.pdf == 0.0f || cblack(ls.L)) continue;
                const Material& m    = sc.materials[is.material];
                const int       base = (m.kind == SP_MAT_CLEARCOAT) ? sc.materials[m.base].kind : m.kind;
                if (base == SP_MAT_LAMBERTIAN) continue;
                const Onb o = onb_from_v(is.n, l.q);
                if (to_onb(o, wo).y != 0.0f) rng_skip(rng, 32);
            }
        }
    }
}

// ------------------------------------------------------------------------- chunked shading
template <int MINW>
__global__ void __launch_bounds__(64 * WAVES_PER_BLOCK, MINW) ck_shade(Scene sc, ChunkArgs a)
{
    extern __shared__ uint32_t lds[];
    const Lds      l     = lds_setup(sc, lds, true);
    const uint32_t lane  = threadIdx.x & 63u;
    Rng            rng;
    uint64_t       shadow_total = 0, draws_total = 0;
    while (true) {
        const int64_t item = grab(a.counter + 1);
        if (item >= a.num_tiles * (int64_t)a.chunks) break;
        // a tile's chunks are adjacent in the queue, so a slow tile's chunks run side by side
        const int64_t  slot = item / a.chunks;
        const uint32_t c    = (uint32_t)(item % a.chunks);
        const Px       px   = pixel(sc, a, slot, lane);
        const size_t   p    = (size_t)slot * 64 + lane;
        const uint32_t i0   = c * a.chunk_len;
        const uint32_t i1   = min(a.spp, i0 + a.chunk_len);
        if (px.inside && i0 < i1) {
        // every generation this chunk draws from was written by ck_count: read-only stream
        const uint32_t st = a.snap_ctl[(size_t)c * a.n_px + p];
        rng.base  = a.gens + (size_t)slot * a.gens_per_px * MT_GEN_WORDS + (size_t)lane * MT_BLK;
        rng.idx   = (int)(st & 0xffffu);
        rng.cur   = (int)(st >> 16);
        rng.lin   = 1;
        rng.pre   = 1;
        rng.ready = 1;
        rng.draws = 0;
        rng.pfn   = 0;
        Ctx ctx{ sc, rng, l.q, l.st, 0u, 0u };
        for (uint32_t i = i0; i < i1; ++i) {
            rng_prepare(rng);
            const float4   rec  = a.hits[(size_t)i * a.n_px + p];
            const uint32_t code = __float_as_uint(rec.y);
            if (code == NO_HIT) continue; // miss or light-only hit: L was stored by ck_camera
            const Ray   ray = camera_ray_px(sc, px, i, l.q);
            const Hit   h{ rec.x, code, rec.z, rec.w };
            const Isect is  = finish_hit(sc, h, ray, l.q);
            const rgb   L   = direct_nee(ctx, is, neg(ray.d));
            a.L[((size_t)i * 3 + 0) * a.n_px + p] = L.r;
            a.L[((size_t)i * 3 + 1) * a.n_px + p] = L.g;
            a.L[((size_t)i * 3 + 2) * a.n_px + p] = L.b;
        }
        shadow_total += ctx.shadow;
        draws_total += rng.draws;
        }
    }
    wave_add(a.counters + 1, shadow_total);
    wave_add(a.counters + 3, draws_total);
}

// ------------------------------------------------------------------------------ resolve
__global__ void __launch_bounds__(256) ck_sum(Scene sc, ChunkArgs a)
{
    const int64_t p = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (p >= (int64_t)a.n_px) return;
    const Px px  = pixel(sc, a, p >> 6, (uint32_t)p & 63u);
    rgb      acc = mkc(0, 0, 0);
    if (px.inside) {
        for (uint32_t i = 0; i < a.spp; ++i)
            acc = cadd(acc, mkc(a.L[((size_t)i * 3 + 0) * a.n_px + p], a.L[((size_t)i * 3 + 1) * a.n_px + p],
                                a.L[((size_t)i * 3 + 2) * a.n_px + p])); // image(p) += integrate(...)
        acc = cdivs(acc, (float)a.spp);                                    // image(p) /= num_pixel_samples
    }
    const int64_t o = (a.slot_map ? (int64_t)a.slot_map[p >> 6] : (p >> 6)) * 64 + (p & 63);
    a.out[(size_t)o * 3 + 0] = acc.r;
    a.out[(size_t)o * 3 + 1] = acc.g;
    a.out[(size_t)o * 3 + 2] = acc.b;
}

// ck_shade occupancy: 4 waves per SIMD (128 VGPRs, ~116 B spill).  Bunny 8-way shard per GPU:
// 1686 / 2039 / 2161 Mrays/s at 2 / 3 / 4 waves (profiles/r02/s5): the chunk kernel's lanes wait
// on generator-store loads, and more waves hide them better than fewer spills do.
typedef void (*CkShadeFn)(Scene, ChunkArgs);
static CkShadeFn shade_kernel() { return ck_shade<4>; }

int chunk_blocks_per_cu(size_t lds_bytes)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, shade_kernel(), 64 * WAVES_PER_BLOCK, lds_bytes) != hipSuccess) return 1;
    return n > 0 ? n : 1;
}

hipError_t chunk_camera(const Scene& sc, const ChunkArgs& a, int n_cu, hipStream_t stream)
{
    const size_t rs_bytes    = (size_t)rsqrt_words(sc) * 4;
    const size_t stack_bytes = (size_t)WAVES_PER_BLOCK * sc.stack_words * 64 * 4;
    const int64_t cam_waves  = a.num_tiles * (int64_t)a.spp;
    int           cam_per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&cam_per_cu, ck_camera, 64 * WAVES_PER_BLOCK, rs_bytes + stack_bytes) !=
            hipSuccess || cam_per_cu < 1)
        cam_per_cu = 1;
    const int64_t cam_blocks = std::max<int64_t>(1, std::min<int64_t>((cam_waves + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK,
                                                                      (int64_t)cam_per_cu * std::max(1, n_cu)));
    hipLaunchKernelGGL(ck_camera, dim3((unsigned)cam_blocks), dim3(64 * WAVES_PER_BLOCK), rs_bytes + stack_bytes, stream, sc, a);
    return hipGetLastError();
}

hipError_t chunk_render(const Scene& sc, const ChunkArgs& a, int persistent_blocks, int n_cu, hipStream_t stream)
{
    const size_t rs_bytes    = (size_t)rsqrt_words(sc) * 4;
    const size_t stack_bytes = (size_t)WAVES_PER_BLOCK * sc.stack_words * 64 * 4;
    const int64_t cam_waves  = a.num_tiles * (int64_t)a.spp;
    int           cam_per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&cam_per_cu, ck_camera, 64 * WAVES_PER_BLOCK, rs_bytes + stack_bytes) !=
            hipSuccess || cam_per_cu < 1)
        cam_per_cu = 1;
    const int64_t cam_blocks = std::max<int64_t>(1, std::min<int64_t>((cam_waves + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK,
                                                                      (int64_t)cam_per_cu * std::max(1, n_cu)));
    hipLaunchKernelGGL(ck_camera, dim3((unsigned)cam_blocks), dim3(64 * WAVES_PER_BLOCK), rs_bytes + stack_bytes, stream, sc, a);
    hipError_t e = hipGetLastError();
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(ck_count, dim3((unsigned)((a.num_tiles + WAVES_PER_BLOCK - 1) / WAVES_PER_BLOCK)),
                       dim3(64 * WAVES_PER_BLOCK), rs_bytes, stream, sc, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    hipLaunchKernelGGL(shade_kernel(), dim3((unsigned)persistent_blocks), dim3(64 * WAVES_PER_BLOCK), rs_bytes + stack_bytes,
                       stream, sc, a);
    if ((e = hipGetLastError()) != hipSuccess) return e;
    return chunk_sum(sc, a, stream);
}

hipError_t chunk_sum(const Scene& sc, const ChunkArgs& a, hipStream_t stream)
{
    hipLaunchKernelGGL(ck_sum, dim3((unsigned)((a.n_px + 255) / 256)), dim3(256), 0, stream, sc, a);
    return hipGetLastError();
}

} // namespace spd
