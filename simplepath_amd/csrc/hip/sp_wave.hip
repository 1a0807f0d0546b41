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
#include "sp_path.hpp"
#include "sp_wave.hpp"

namespace spd {

constexpr int WF_BLOCK = 256;

struct PixelRef {
    uint32_t px, py;
    bool     inside;
};

__device__ __forceinline__ PixelRef pixel_of(const Scene& sc, const WaveArgs& w, int64_t p)
{
    const int64_t  slot = p >> 6;
    const uint32_t lane = (uint32_t)p & 63u;
    const int32_t  tile = w.tile_ids ? w.tile_ids[slot] : (int32_t)slot;
    PixelRef       r;
    r.px     = (uint32_t)((tile % w.tiles_x) * 8) + morton_decode_1(lane);
    r.py     = (uint32_t)((tile / w.tiles_x) * 8) + morton_decode_1(lane >> 1);
    r.inside = (int)r.px < sc.width && (int)r.py < sc.height;
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

__device__ __forceinline__ void wave_count(unsigned long long* ctr, uint32_t v)
{
    unsigned long long s = v;
    for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
    if ((threadIdx.x & 63) == 0 && s) atomicAdd(ctr, s);
}

__device__ __forceinline__ Rng rng_load(const WaveArgs& w, int64_t p)
{
    Rng            r;
    const uint32_t st = w.rstate[p];
    r.base  = w.mt_state + (size_t)(p >> 6) * (2 * MT_N * 64) + (p & 63);
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
    const int64_t p = (int64_t)blockIdx.x * WF_BLOCK + threadIdx.x;
    if (p >= w.n) return;
    const PixelRef pr = pixel_of(sc, w, p);
    w.acc[p] = 0.0f;
    w.acc[w.n + p] = 0.0f;
    w.acc[2 * w.n + p] = 0.0f;
    if (!pr.inside) {
        w.rstate[p] = 0;
        return;
    }
    Rng r;
    r.base = w.mt_state + (size_t)(p >> 6) * (2 * MT_N * 64) + (p & 63);
    rng_seed(r, ((pr.px << 16u) | pr.py) ^ 0xb0ae9d99u); // get_integrator_sampler (main.cpp:73)
    rng_store(w, p, r);
}

// Primary query: Integrator::integrate's intersect_lights + intersect (Integrator.cpp:277-283).
__global__ void __launch_bounds__(WF_BLOCK) wf_primary(Scene sc, WaveArgs w, uint32_t sample)
{
    extern __shared__ uint32_t lds[];
    const int64_t p    = (int64_t)blockIdx.x * WF_BLOCK + threadIdx.x;
    const int     lane = threadIdx.x & 63;
    if (blockIdx.x == 0 && threadIdx.x == 0) *w.qcount = 0u; // wf_shadow of the previous sample is done
    if (p >= w.n) return;
    const PixelRef pr = pixel_of(sc, w, p);
    float4         hrec = make_float4(0.0f, __uint_as_float(0xffffffffu), 0.0f, 0.0f);
    uint32_t       rays = 0, hits = 0;
    if (pr.inside && sc.max_depth > 0) {
        const Rsq   q{ sc.rsqrt_entries, sc.rsqrt_bits, sc.rsqrt_zero, sc.rsqrt_denorm };
        const Stack st{ lds + (threadIdx.x >> 6) * sc.stack_depth * 64, lane };
        const Ray   ray = camera_ray(sc, pr, sample, q);
        rays            = 1;
        float          tmax = k_infinite;
        const LightHit lh   = scene_intersect_lights(sc, ray, k_ray_epsilon, tmax, st);
        if (lh.hit) tmax = lh.t;
        const Hit h = scene_intersect(sc, ray, k_ray_epsilon, tmax, st);
        if (h.code != 0xffffffffu) {
            hrec = make_float4(h.t, __uint_as_float(h.code), h.beta, h.gamma);
            hits = 1;
        } else if (lh.hit) {
            const rgb L = cadd(mkc(0, 0, 0), cmul(mkc(1, 1, 1), lh.L));
            w.acc[p]           = w.acc[p] + L.r;
            w.acc[w.n + p]     = w.acc[w.n + p] + L.g;
            w.acc[2 * w.n + p] = w.acc[2 * w.n + p] + L.b;
        }
    }
    w.hit[p] = hrec;
    wave_count(w.counters + 0, rays);
    wave_count(w.counters + 4, hits);
}

// Shading: direct_nee's sampling half (Integrator.cpp:287-296).
__global__ void __launch_bounds__(WF_BLOCK) wf_shade(Scene sc, WaveArgs w, uint32_t sample)
{
    extern __shared__ uint32_t lds[];
    const int rs_words = 2 << sc.rsqrt_bits;
    for (int i = threadIdx.x; i < rs_words; i += WF_BLOCK) lds[i] = sc.rsqrt_entries[i];
    __syncthreads();
    const int64_t p = (int64_t)blockIdx.x * WF_BLOCK + threadIdx.x;
    if (p >= w.n) return;
    const PixelRef pr = pixel_of(sc, w, p);
    uint32_t       mask = 0, draws = 0;
    if (pr.inside) {
        const Rsq q{ lds, sc.rsqrt_bits, sc.rsqrt_zero, sc.rsqrt_denorm };
        Rng       rng = rng_load(w, p);
        rng_prepare(rng);
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
            for (int li = 0; li < sc.n_lights; ++li) {
                const Light&  l  = sc.lights[li];
                const LSample ls = light_sample(l, is.p, is.n, next2D(rng), q);
                if (ls.pdf == 0.0f || cblack(ls.L)) continue;
                const f3  wi = ls.ray.d;
                const rgb f  = material_eval(sc, is.material, wo, wi, is.n, rng, q);
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
    // active-ray compaction: wave ballot + one atomic per wave, queue keeps pixel order in a wave
    const unsigned long long ballot = __ballot(mask != 0);
    if (ballot) {
        const int      lane   = threadIdx.x & 63;
        const uint32_t total  = (uint32_t)__popcll(ballot);
        uint32_t       base   = 0;
        if (lane == 0) base = atomicAdd(w.qcount, total);
        base = __shfl(base, 0, 64);
        if (mask) w.queue[base + (uint32_t)__popcll(ballot & ((1ull << lane) - 1ull))] = (uint32_t)p;
    }
    wave_count(w.counters + 3, draws);
}

// Shadow queries + accumulation: direct_nee's occlusion half (Integrator.cpp:297-300).
__global__ void __launch_bounds__(WF_BLOCK) wf_shadow(Scene sc, WaveArgs w)
{
    extern __shared__ uint32_t lds[];
    const int      lane  = threadIdx.x & 63;
    const Stack    st{ lds + (threadIdx.x >> 6) * sc.stack_depth * 64, lane };
    const uint32_t count = *w.qcount;
    uint32_t       shadow = 0;
    for (uint32_t k = blockIdx.x * WF_BLOCK + threadIdx.x; k < count; k += gridDim.x * WF_BLOCK) {
        const int64_t  p    = w.queue[k];
        const float4   o    = w.shp[p];
        const uint32_t mask = __float_as_uint(o.w);
        rgb            L    = mkc(0, 0, 0);
        for (uint32_t m = mask; m; m &= m - 1) {
            const int     li = __ffs(m) - 1;
            const float4* e  = w.sh + ((size_t)li * w.n + p) * 2;
            const float4  d  = e[0];
            const float4  c  = e[1];
            Ray           r;
            r.o = mk(o.x, o.y, o.z);
            r.d = mk(d.x, d.y, d.z);
            ++shadow;
            if (!scene_any(sc, r, d.w, c.w, st)) L = cadd(L, mkc(c.x, c.y, c.z));
        }
        w.acc[p]           = w.acc[p] + L.r;
        w.acc[w.n + p]     = w.acc[w.n + p] + L.g;
        w.acc[2 * w.n + p] = w.acc[2 * w.n + p] + L.b;
    }
    wave_count(w.counters + 0, shadow); // occluded() counts the query as a ray too
    wave_count(w.counters + 1, shadow);
}

__global__ void __launch_bounds__(WF_BLOCK) wf_resolve(Scene sc, WaveArgs w, float* out)
{
    const int64_t p = (int64_t)blockIdx.x * WF_BLOCK + threadIdx.x;
    if (p >= w.n) return;
    const PixelRef pr = pixel_of(sc, w, p);
    rgb            a  = mkc(w.acc[p], w.acc[w.n + p], w.acc[2 * w.n + p]);
    if (pr.inside) a = cdivs(a, (float)w.spp); // image(p) /= num_pixel_samples (main.cpp:102)
    float* o = out + (size_t)p * 3;
    o[0]     = a.r;
    o[1]     = a.g;
    o[2]     = a.b;
    wave_count(w.counters + 2, pr.inside ? w.spp : 0u);
}

// ---------------------------------------------------------------------------- host side
size_t wave_bytes_per_pixel(int n_lights)
{
    return 3 * 4 + 4 + 16 + 16 + (size_t)n_lights * 32 + 4 + 2 * MT_N * 8;
}

hipError_t wave_render(const Scene& sc, const WaveArgs& w, float* out, int traverse_blocks_per_cu, int n_cu,
                       hipStream_t stream, hipEvent_t* ev)
{
    int  e    = 0;
    auto mark = [&]() {
        if (ev) (void)hipEventRecord(ev[e++], stream);
    };
    const unsigned grid      = (unsigned)((w.n + WF_BLOCK - 1) / WF_BLOCK);
    const size_t   stack_lds = (size_t)(WF_BLOCK / 64) * sc.stack_depth * 64 * 4;
    const size_t   rs_lds    = (size_t)(2 << sc.rsqrt_bits) * 4;
    // the shadow queue never exceeds n: a persistent grid sized to fill the chip
    const unsigned sgrid = (unsigned)std::max<int64_t>(1, std::min<int64_t>(grid, (int64_t)n_cu * traverse_blocks_per_cu));
    mark();
    hipLaunchKernelGGL(wf_init, dim3(grid), dim3(WF_BLOCK), 0, stream, sc, w);
    mark();
    for (uint32_t i = 0; i < w.spp; ++i) {
        hipLaunchKernelGGL(wf_primary, dim3(grid), dim3(WF_BLOCK), stack_lds, stream, sc, w, i);
        mark();
        hipLaunchKernelGGL(wf_shade, dim3(grid), dim3(WF_BLOCK), rs_lds, stream, sc, w, i);
        mark();
        hipLaunchKernelGGL(wf_shadow, dim3(sgrid), dim3(WF_BLOCK), stack_lds, stream, sc, w);
        mark();
    }
    hipLaunchKernelGGL(wf_resolve, dim3(grid), dim3(WF_BLOCK), 0, stream, sc, w, out);
    mark();
    return hipGetLastError();
}

int wave_traverse_blocks_per_cu(const Scene& sc)
{
    const size_t stack_lds = (size_t)(WF_BLOCK / 64) * sc.stack_depth * 64 * 4;
    int          n         = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, wf_shadow, WF_BLOCK, stack_lds) != hipSuccess) return 1;
    return n > 0 ? n : 1;
}

} // namespace spd
