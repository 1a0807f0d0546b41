// sp_mega.hpp -- megakernel form of the per-pixel path: one lane owns one pixel for all its
// samples (main.cpp:94-102).  Used for the multi-bounce integrators and as the comparison point
// for the wavefront pipeline (sp_wave.hip).  Instantiated per integrator in sp_mega_*.hip so the
// heavy translation units compile in parallel.
#pragma once
#include "sp_path.hpp"

namespace spd {
inline namespace SPD_LAYOUT_NS {

constexpr int WAVES_PER_BLOCK = 4;

template <int INTEG>
__device__ __forceinline__ rgb integrate(Ctx& c, Ray ray)
{
    if constexpr (INTEG == SP_INTEGRATOR_BRUTE_FORCE) return integrate_bruteforce(c, ray);
    else if constexpr (INTEG == SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE) return integrate_iterative<false>(c, ray);
    else if constexpr (INTEG == SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE_RR) return integrate_iterative<true>(c, ray);
    else if constexpr (INTEG == SP_INTEGRATOR_ITERATIVE_RRNEE) return integrate_rrnee(c, ray);
    else if constexpr (INTEG == SP_INTEGRATOR_WHITTED) return integrate_whitted(c, ray);
    else return integrate_direct(c, ray);
}

// ------------------------------------------------------------------------------ tail chunks
// (RenderArgs::tail, sp_device.hpp).  Why: a tile's 64 pixels run their 256-sample stream chains in
// one wave, so the frame's last work items are whole tiles, whose durations move by ~20 % with
// what the other waves on their SIMD do -- no cost estimate can order that noise away (DESIGN.md
// §11l: bunny ends at 262.2 ms against 246.5 ms of work per wave).  The K most expensive tiles are
// cut into sample chunks (the sample-chunk pipeline's scheme, sp_chunk.hip) whose shading comes
// last in the queue, where short items fill the waves that would otherwise idle.  Same stream words
// and floating-point sequence per sample, and the samples are summed in order (chunk_sum): the
// image and the ray / draw counts are the megakernel's bit for bit.

// PerspectiveCamera::generate_ray_impl of sample i (the sample loop below and sp_chunk.hip)
__device__ __forceinline__ Ray tail_camera_ray(const Scene& sc, uint32_t px, uint32_t py, uint32_t i, const Rsq& q)
{
    const uint32_t seed2d = ((px << 16u) | py) ^ 0x6184faf4u;
    const float    sx     = rseq_component(seed2d, sc.alpha2_0, i);
    const float    sy     = rseq_component(seed2d, sc.alpha2_1, i);
    const float    fx     = (float)(int)px + sx;
    const float    fy     = (float)(int)py + sy;
    Ray            ray;
    ray.o = sc.camera.p;
    ray.d = normalize(add(add(scale(fx, sc.camera.vx), scale(fy, sc.camera.vy)), sc.camera.vz), q);
    return ray;
}

// Camera item c of the fused queue (TailArgs::n_cam): samples [b cam_block, (b + 1) cam_block) of
// list slot c / blocks -- sp_chunk.hip ck_camera's work for them (Integrator.cpp:277-283: intersect
// lights, then geometry; the hit record, a light-only hit's radiance, the sample's draw count) --
// then an agent-scope release and cam_done[slot] += samples done (the slot's prep waits for spp).
__device__ __forceinline__ void fused_camera(const Scene& sc, const RenderArgs& args, const Rsq& q, Stack& st, int64_t c,
                                             uint32_t lane, uint32_t dx, uint32_t dy)
{
    const TailArgs& ta     = *args.tail;
    const int64_t   nb     = (args.spp + ta.cam_block - 1) / ta.cam_block;
    const int64_t   slot   = c / nb;
    const uint32_t  i0     = (uint32_t)(c % nb) * ta.cam_block;
    const uint32_t  i1     = min(args.spp, i0 + ta.cam_block);
    const int32_t   tile   = args.tile_ids ? args.tile_ids[slot] : (int32_t)slot;
    const uint32_t  px     = (uint32_t)((tile % args.tiles_x) * 8) + dx;
    const uint32_t  py     = (uint32_t)((tile / args.tiles_x) * 8) + dy;
    const bool      inside = px < (uint32_t)sc.width && py < (uint32_t)sc.height;
    const size_t    p      = (size_t)slot * 64 + lane;
    for (uint32_t i = i0; i < i1; ++i) {
        float4   rec   = make_float4(0.0f, __uint_as_float(0xffffffffu), 0.0f, 0.0f);
        rgb      L     = mkc(0, 0, 0);
        uint32_t ndraw = 0;
        if (inside && sc.max_depth > 0) {
            const Ray      ray = tail_camera_ray(sc, px, py, i, q);
            const LightHit lh  = scene_intersect_lights(sc, ray, k_ray_epsilon, k_infinite, st);
            const Hit      h   = scene_intersect(sc, ray, k_ray_epsilon, lh.hit ? lh.t : k_infinite, st);
            if (h.code != 0xffffffffu) {
                rec   = make_float4(h.t, __uint_as_float(h.code), h.beta, h.gamma);
                ndraw = sample_draws(sc, finish_hit(sc, h, ray, q), neg(ray.d), q);
            } else if (lh.hit) {
                L = cadd(L, cmul(mkc(1, 1, 1), light_hit_L(sc, lh, ray.d, q)));
            }
        }
        ta.draws_out[(size_t)i * ta.n_px + p]      = (uint16_t)ndraw;
        ta.hits[(size_t)i * ta.n_px + p]           = rec;
        ta.L[((size_t)i * 3 + 0) * ta.n_px + p] = L.r;
        ta.L[((size_t)i * 3 + 1) * ta.n_px + p] = L.g;
        ta.L[((size_t)i * 3 + 2) * ta.n_px + p] = L.b;
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_fetch_add(ta.cam_done + slot, i1 - i0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Prep item k (queue item k < K): tile order[k]'s camera rays (Integrator.cpp:277-283: intersect
// lights, then geometry) for every sample, their hit records and the radiance of light-only hits;
// each sample's draw count (sample_draws) summed into the stream position at every chunk start;
// then every generation of each pixel's stream, twisted once, into the store (sp_chunk.hip ck_camera
// + ck_count in one item).  Publishes the store with an agent-scope release before setting
// ready[k] (MI355X guide: stores, vmcnt(0), release, vmcnt(0), flag).
// DRAWS: the sample-chunk pipeline's fused form (TailArgs::draws from ck_camera, no camera rays here).
// REPLAY: an image light's counts, replayed on the stream (TailArgs::replay; sp_tail_kernel<., true>).
template <bool DRAWS, bool REPLAY = false>
__device__ __forceinline__ void tail_prep(const Scene& sc, const RenderArgs& args, const Rsq& q, Stack& st, int64_t k,
                                          uint32_t lane, uint32_t dx, uint32_t dy, uint32_t& rays_total,
                                          uint32_t& samples_total)
{
    const TailArgs& ta     = *args.tail;
    const int64_t   slot   = args.order ? args.order[k] : k;
    const int32_t   tile   = args.tile_ids ? args.tile_ids[slot] : (int32_t)slot;
    const uint32_t  px     = (uint32_t)((tile % args.tiles_x) * 8) + dx;
    const uint32_t  py     = (uint32_t)((tile / args.tiles_x) * 8) + dy;
    const bool      inside = px < (uint32_t)sc.width && py < (uint32_t)sc.height;
    const size_t    p      = (size_t)k * 64 + lane;
    Rng             rng;
    rng.lin   = 1; // generation g in buffer g of the pixel's store
    rng.base  = ta.gens + (size_t)k * ta.gens_per_px * MT_GEN_WORDS + (size_t)lane * MT_BLK;
    rng.cur   = 0; // (a pixel outside the image keeps this state; its chunks never run)
    rng.idx   = MT_N;
    rng.ready = 0;
    rng.draws = 0;
    // main.cpp:73; generation 0 (the seeded state) is never drawn from: the seed writes generation 1
    if (inside) rng_seed_twisted(rng, ((px << 16u) | py) ^ 0xb0ae9d99u);
    uint32_t T = 0; // stream position (words drawn) before sample i
    if constexpr (DRAWS) {
        if (ta.n_cam > 0) { // the camera items of this slot (all taken before any prep) have finished
            if (lane == 0)
                while (__hip_atomic_load(ta.cam_done + slot, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) < args.spp)
                    __builtin_amdgcn_s_sleep(2);
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
        // the sample-chunk pipeline's form: counts from ck_camera, summed in batches of loads that
        // are all in flight together (sp_chunk.hip ck_count)
        const uint16_t* dp = ta.draws + p;
        for (uint32_t i0 = 0; i0 < args.spp; i0 += 8) {
            uint32_t d[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) d[j] = (inside && i0 + j < args.spp) ? (uint32_t)dp[(size_t)(i0 + j) * ta.n_px] : 0u;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const uint32_t i = i0 + (uint32_t)j;
                if (i < args.spp && i % ta.chunk_len == 0) {
                    const uint32_t g = T ? (T - 1) / MT_N + 1 : 0u;
                    const uint32_t w = T ? T - (g - 1) * MT_N : (uint32_t)MT_N;
                    ta.snap_ctl[(size_t)(i / ta.chunk_len) * ta.n_px + p] = w | (g << 16);
                }
                T += d[j];
            }
        }
    } else {
    constexpr bool replay = REPLAY;
    for (uint32_t i = 0; i < args.spp; ++i) {
        if (i % ta.chunk_len == 0) {
            uint32_t snap;
            if (replay) { // the replayed stream's own position (sp_chunk.hip ck_count)
                snap = (uint32_t)rng.idx | ((uint32_t)rng.cur << 16);
            } else { // the lazy-switch form rng_skip leaves (sp_chunk.hip ck_count)
                const uint32_t g = T ? (T - 1) / MT_N + 1 : 0u;
                const uint32_t w = T ? T - (g - 1) * MT_N : (uint32_t)MT_N;
                snap             = w | (g << 16);
            }
            ta.snap_ctl[(size_t)(i / ta.chunk_len) * ta.n_px + p] = snap;
        }
        if (replay && inside) rng_prepare(rng);
        float4   rec = make_float4(0.0f, __uint_as_float(0xffffffffu), 0.0f, 0.0f);
        rgb      L   = mkc(0, 0, 0);
        uint32_t nd  = 0;
        if (inside && sc.max_depth > 0) {
            const Ray      ray = tail_camera_ray(sc, px, py, i, q);
            const LightHit lh  = scene_intersect_lights(sc, ray, k_ray_epsilon, k_infinite, st);
            const Hit      h   = scene_intersect(sc, ray, k_ray_epsilon, lh.hit ? lh.t : k_infinite, st);
            if (h.code != 0xffffffffu) {
                rec = make_float4(h.t, __uint_as_float(h.code), h.beta, h.gamma);
                const Isect is = finish_hit(sc, h, ray, q);
                if (!replay) {
                    nd = sample_draws(sc, is, neg(ray.d), q);
                } else { // direct_nee's draws: Light::sample, then the glossy estimate of a usable sample
                    const f3 wo = neg(ray.d);
                    for (int li = 0; li < sc.n_lights; ++li) {
                        const Light   lt = uload_light(sc.lights + li);
                        const LSample ls = light_sample(sc, lt, is.p, is.n, next2D(rng), q);
                        if (ls.pdf == 0.0f || cblack(ls.L)) continue;
                        const Material& m    = sc.materials[is.material];
                        const int       base = (m.kind == SP_MAT_CLEARCOAT) ? sc.materials[m.base].kind : m.kind;
                        if (base == SP_MAT_LAMBERTIAN) continue;
                        const Onb o = onb_from_v(is.n, q);
                        if (to_onb(o, wo).y != 0.0f) rng_skip(rng, 32);
                    }
                }
            } else if (lh.hit) {
                L = cadd(L, cmul(mkc(1, 1, 1), light_hit_L(sc, lh, ray.d, q)));
            }
        }
        ta.hits[(size_t)i * ta.n_px + p]          = rec;
        ta.L[((size_t)i * 3 + 0) * ta.n_px + p] = L.r;
        ta.L[((size_t)i * 3 + 1) * ta.n_px + p] = L.g;
        ta.L[((size_t)i * 3 + 2) * ta.n_px + p] = L.b;
        T += nd;
    }
    }
    if (inside) {
        // (the replay twisted each generation as its draws reached it)
        const uint32_t G = T ? (T - 1) / MT_N + 1 : 0u;
#pragma unroll 1
        for (uint32_t g = 1; g < G; ++g) mt_twist_blocked<SP_TWIST_SKIP_BLOCK>(mt_buf(rng, (int)g), mt_buf(rng, (int)g + 1));
        if constexpr (!DRAWS) { // (the sample-chunk pipeline counts camera rays and samples on the host)
            if (sc.max_depth > 0) rays_total += args.spp; // the camera rays (trace() counts them)
            samples_total += args.spp;
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) __hip_atomic_store(ta.ready + k, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

// Chunk item j (queue item num_tiles + j): samples [c len, (c + 1) len) of tile order[k], k = j /
// chunks, from the chunk's stream position in the store (no twisting: every generation is there),
// direct_nee on the stored hit (sp_chunk.hip ck_shade); each sample's radiance into L.  Waits for
// prep item k (taken before any chunk item: the queue is one counter, so its wave is running).
__device__ __forceinline__ void tail_chunk(const Scene& sc, const RenderArgs& args, const Rsq& q, Stack& st, int64_t j,
                                           uint32_t lane, uint32_t dx, uint32_t dy, uint32_t& rays_total,
                                           uint32_t& shadow_total, uint32_t& draws_total)
{
    const TailArgs& ta = *args.tail;
    const int64_t   k  = j / ta.chunks;
    const uint32_t  c  = (uint32_t)(j % ta.chunks);
    if (lane == 0)
        while (__hip_atomic_load(ta.ready + k, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == 0u) __builtin_amdgcn_s_sleep(4);
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const int64_t  slot   = args.order ? args.order[k] : k;
    const int32_t  tile   = args.tile_ids ? args.tile_ids[slot] : (int32_t)slot;
    const uint32_t px     = (uint32_t)((tile % args.tiles_x) * 8) + dx;
    const uint32_t py     = (uint32_t)((tile / args.tiles_x) * 8) + dy;
    const bool     inside = px < (uint32_t)sc.width && py < (uint32_t)sc.height;
    const size_t   p      = (size_t)k * 64 + lane;
    const uint32_t i0     = c * ta.chunk_len;
    const uint32_t i1     = min(args.spp, i0 + ta.chunk_len);
    if (!inside || i0 >= i1) return;
    const uint32_t snap = ta.snap_ctl[(size_t)c * ta.n_px + p];
    Rng            rng;
    rng.base  = ta.gens + (size_t)k * ta.gens_per_px * MT_GEN_WORDS + (size_t)lane * MT_BLK;
    rng.idx   = (int)(snap & 0xffffu);
    rng.cur   = (int)(snap >> 16);
    rng.lin   = 1;
    rng.pre   = 1; // every generation is in the store: a buffer switch never twists
    rng.ready = 1;
    rng.draws = 0;
    rng.pfn   = 0;
    Ctx ctx{ sc, rng, q, st, 0u, 0u };
    for (uint32_t i = i0; i < i1; ++i) {
        rng_prepare(rng);
        const float4   rec  = ta.hits[(size_t)i * ta.n_px + p];
        const uint32_t code = __float_as_uint(rec.y);
        if (code == 0xffffffffu) continue; // miss or light-only hit: L was stored by the prep item
        const Ray   ray = tail_camera_ray(sc, px, py, i, q);
        const Hit   h{ rec.x, code, rec.z, rec.w };
        const Isect is  = finish_hit(sc, h, ray, q);
        const rgb   L   = direct_nee(ctx, is, neg(ray.d));
        ta.L[((size_t)i * 3 + 0) * ta.n_px + p] = L.r;
        ta.L[((size_t)i * 3 + 1) * ta.n_px + p] = L.g;
        ta.L[((size_t)i * 3 + 2) * ta.n_px + p] = L.b;
    }
    rays_total += ctx.rays;
    shadow_total += ctx.shadow;
    draws_total += rng.draws;
}

// Persistent kernel: 4 waves per block share the LDS RSQRTSS table; each wave independently
// pulls 8x8 tiles from the queue (TileScheduler::get_next_tile) and owns one MT state slot.
// One instantiation per integrator so each carries only its own live state; MINW is the
// __launch_bounds__ occupancy request (waves per SIMD) chosen by measurement.
// PROBE: the tile-order probe pass (sp_mega.hip) -- the same code writing each tile's wave time
// to args.tile_time instead of radiance, compiled as its own kernel (sp_probe_kernel) so that
// profiles list the probe and the render apart.
// TAIL: 1 the DirectLighting render with tail chunks (sp_tail_kernel; queue layout in TailArgs; 3:
// the same with an image light, its preps replaying Light::sample), 2 the sample-chunk pipeline's
// fused form (preps from ck_camera's counts interleaved with the chunks, no whole tiles:
// sp_fused_kernel).  One kernel per form, so each carries only its own code.
template <int INTEG, bool PROBE, int TAIL = 0>
__device__ __forceinline__ void render_tiles_body(const Scene& sc, const RenderArgs& args)
{
    extern __shared__ uint32_t lds[];
    const int tid  = threadIdx.x;
    const int lane = tid & 63;
    const int wave = tid >> 6;
    const int rs_words = rsqrt_words(sc);
    for (int i = tid; i < rs_words; i += 64 * WAVES_PER_BLOCK) lds[i] = sc.rsqrt_entries[i];
    libm_lds_init(tid, 64 * WAVES_PER_BLOCK);
#ifdef SP_WAVE_PROF
    if (lane < 16) wprof_lds[wave * 16 + lane] = 0;
#endif
#ifdef SP_TRAFFIC_DIAG
    if (lane < 32) tdg_lds[wave * 32 + lane] = 0;
#endif
    __syncthreads();
    Rsq   q{ lds };
    Stack st{ lds + rs_words + wave * sc.stack_words * 64, lane, sc.stack_depth };

    const size_t gwave = (size_t)blockIdx.x * WAVES_PER_BLOCK + wave;
    Rng          rng;
    rng.base = args.mt_state + gwave * (2 * (size_t)MT_GEN_WORDS) + (size_t)lane * MT_BLK;

    uint32_t rays_total = 0, shadow_total = 0, samples_total = 0, draws_total = 0;
    // The probe's tile times are timer readings (run-to-run noise) and only order the queue, so
    // its draws need not be the pixels' own streams: each lane seeds once and its stream runs on
    // across the wave's tiles, instead of a 312-word seed and a first twist per tile.
    if constexpr (PROBE) rng_seed(rng, (uint32_t)(gwave * 64 + lane) ^ 0xb0ae9d99u);
    const uint32_t dx = morton_decode_1((uint32_t)lane);
    const uint32_t dy = morton_decode_1((uint32_t)lane >> 1);
    while (true) {
        int grabbed = 0;
        if (lane == 0) grabbed = atomicAdd(args.tile_counter, 1);
        const int64_t item = __shfl(grabbed, 0, 64);
        if constexpr (TAIL == 2) {
            { // every tile cut: [camera items] then the preps interleaved with the chunks
                const int64_t NC = args.tail_cam;
                if (item < NC) {
                    fused_camera(sc, args, q, st, item, (uint32_t)lane, dx, dy);
                    continue;
                }
                const int64_t it = item - NC;
                const int64_t K = args.tail_prep, C = args.tail_items / max<int64_t>(1, K), P = min(args.tail_front, K);
                if (it >= K + args.tail_items) break;
                int64_t   idx  = it;
                bool      prep = it < P;
                if (!prep) {
                    const int64_t j = it - P, full = K - P; // groups 0 .. full - 1: C chunks + prep g + P
                    if (j < full * (C + 1)) {
                        const int64_t g = j / (C + 1), r = j % (C + 1);
                        prep            = r == C;
                        idx             = prep ? g + P : g * C + r;
                    } else {
                        idx = full * C + (j - full * (C + 1)); // the last P tiles' chunks
                    }
                }
                if (prep) tail_prep<true>(sc, args, q, st, idx, (uint32_t)lane, dx, dy, rays_total, samples_total);
                else tail_chunk(sc, args, q, st, idx, (uint32_t)lane, dx, dy, rays_total, shadow_total, draws_total);
                continue;
            }
        } else if constexpr (TAIL == 1 || TAIL == 3) {
            if (item >= args.num_tiles + args.tail_items) break;
            if (item < args.tail_prep) {
                tail_prep<false, TAIL == 3>(sc, args, q, st, item, (uint32_t)lane, dx, dy, rays_total, samples_total);
                continue;
            }
            if (item >= args.num_tiles) {
                tail_chunk(sc, args, q, st, item - args.num_tiles, (uint32_t)lane, dx, dy, rays_total, shadow_total,
                           draws_total);
                continue;
            }
        } else if (item * (PROBE ? (int64_t)args.probe_step : 1) >= args.num_tiles) {
            break;
        }
        const int64_t  slot    = PROBE ? item * args.probe_step : (args.order ? args.order[item] : item);
        const uint64_t t_start = (PROBE || args.tile_diag) ? __builtin_amdgcn_s_memrealtime() : 0;
        const int32_t  tile   = args.tile_ids ? args.tile_ids[slot] : (int32_t)slot;
        const uint32_t px     = (uint32_t)((tile % args.tiles_x) * 8) + dx;
        const uint32_t py     = (uint32_t)((tile / args.tiles_x) * 8) + dy;
        // unsigned compares: a negative tile id (device lists are not checked) lands outside
        const bool     inside = px < (uint32_t)sc.width && py < (uint32_t)sc.height;
        rgb            acc    = mkc(0, 0, 0);
        uint64_t       prof[4] = { 0, 0, 0, 0 };
        if (inside) {
            const uint32_t pix_seed = (px << 16u) | py;
            if constexpr (!PROBE) { // get_integrator_sampler (main.cpp:73)
                if (SP_SEED_FUSED) rng_seed_twisted(rng, pix_seed ^ 0xb0ae9d99u);
                else rng_seed(rng, pix_seed ^ 0xb0ae9d99u);
            }
            const uint32_t seed2d = pix_seed ^ 0x6184faf4u; // RSequenceSampler m_seed_2D (main.cpp:67)
            Ctx c{ sc, rng, q, st, 0u, 0u };
            if (args.deep) {
                c.deep    = args.deep + gwave * 64 + lane;
                c.dstride = args.deep_stride;
            }
            for (uint32_t i = 0; i < args.spp; ++i) {
                rng_prepare(rng);
                // RSequenceSampler::get_next_2D (math/Sampler.h:158) with count i
                const float sx = rseq_component(seed2d, sc.alpha2_0, i);
                const float sy = rseq_component(seed2d, sc.alpha2_1, i);
                const float fx = (float)(int)px + sx;
                const float fy = (float)(int)py + sy;
                // PerspectiveCamera::generate_ray_impl (Cameras/Camera.h:119)
                Ray ray;
                ray.o = sc.camera.p;
                ray.d = normalize(add(add(scale(fx, sc.camera.vx), scale(fy, sc.camera.vy)), sc.camera.vz), q);
                if constexpr (INTEG == SP_INTEGRATOR_MANDELBROT)
                    acc = cadd(acc, integrate_mandelbrot(fx, fy, sc.width, sc.height));
                else
                    SP_WPROF(0, acc = cadd(acc, integrate<INTEG>(c, ray))); // image(p) += integrate(...)
            }
            acc = cdivs(acc, (float)args.spp); // image(p) /= num_pixel_samples
#ifdef SP_MEGA_PROF
            for (int k = 0; k < 4; ++k) prof[k] = c.prof[k];
#endif
            rays_total += c.rays;
            shadow_total += c.shadow;
            samples_total += args.spp;
            draws_total += rng.draws;
        }
        if constexpr (PROBE) { // probe pass (sp_mega.hip tile_order): how long this tile kept the wave
            if (lane == 0) args.tile_time[slot] = (float)(__builtin_amdgcn_s_memrealtime() - t_start);
            continue;
        }
        float* o = args.out + ((size_t)slot * 64 + lane) * 3;
        o[0]     = acc.r;
        o[1]     = acc.g;
        o[2]     = acc.b;
#if !defined(SP_WAVE_PROF) && !defined(SP_TRAFFIC_DIAG) // those builds use the buffer for their totals
        if (args.tile_diag) {
            // {t0, t1, wave, item, then per stage the largest shader-clock total of any lane}
            for (int k = 0; k < 4; ++k)
                for (int off = 32; off > 0; off >>= 1) {
                    const uint64_t o = __shfl_xor(prof[k], off, 64);
                    prof[k]          = o > prof[k] ? o : prof[k];
                }
            const uint64_t t_end  = __builtin_amdgcn_s_memrealtime();
            const uint64_t rec[8] = { t_start, t_end, (uint64_t)gwave, (uint64_t)item, prof[0], prof[1], prof[2], prof[3] };
            if (lane < 8) args.tile_diag[(size_t)slot * 8 + lane] = rec[lane];
        }
#endif
    }
#ifdef SP_WAVE_PROF
    if (args.tile_diag && lane < 16) atomicAdd(args.tile_diag + lane, wprof_lds[wave * 16 + lane]);
#endif
#ifdef SP_TRAFFIC_DIAG
    if (args.tile_diag && lane < 32) atomicAdd(args.tile_diag + 16 + lane, tdg_lds[wave * 32 + lane]);
#endif
    unsigned long long v[4] = { rays_total, shadow_total, samples_total, draws_total };
    for (int k = 0; k < 4; ++k) {
        unsigned long long s = v[k];
        for (int off = 32; off > 0; off >>= 1) s += __shfl_down(s, off, 64);
        if (lane == 0 && s) atomicAdd(args.counters + k, s);
    }
}
template <int INTEG, int MINW>
__global__ void __launch_bounds__(64 * WAVES_PER_BLOCK, MINW) sp_render_kernel(Scene sc, RenderArgs args)
{
    render_tiles_body<INTEG, false>(sc, args);
}
template <int INTEG, int MINW>
__global__ void __launch_bounds__(64 * WAVES_PER_BLOCK, MINW) sp_probe_kernel(Scene sc, RenderArgs args)
{
    render_tiles_body<INTEG, true>(sc, args);
}
template <int MINW, bool REPLAY>
__global__ void __launch_bounds__(64 * WAVES_PER_BLOCK, MINW) sp_tail_kernel(Scene sc, RenderArgs args)
{
    render_tiles_body<SP_INTEGRATOR_DIRECT_LIGHTING, false, REPLAY ? 3 : 1>(sc, args);
}
template <int MINW>
__global__ void __launch_bounds__(64 * WAVES_PER_BLOCK, MINW) sp_fused_kernel(Scene sc, RenderArgs args)
{
    render_tiles_body<SP_INTEGRATOR_DIRECT_LIGHTING, false, 2>(sc, args);
}
} // inline namespace SPD_LAYOUT_NS

using KernelFn = void (*)(Scene, RenderArgs);
KernelFn mega_direct(int variant);
KernelFn mega_iterative(int integ);
KernelFn mega_rrnee(int waves);
KernelFn mega_recursive(int integ);
KernelFn mega_mandelbrot();
KernelFn probe_direct(int variant); // nullptr: no probe kernel (queue order)
KernelFn probe_rrnee(int waves);
KernelFn tail_direct(int variant, bool replay); // DirectLighting with tail chunks, 3 or 4 waves per SIMD
                                                 // (sp_mega_tail.hip; replay: an image light, 4 waves)
KernelFn fused_chunks();           // the sample chunks' fused form, 4 waves per SIMD (sp_mega_tail.hip)
hipError_t launch_tile_order(float* tile_time, int64_t n_tiles, float factor, int tiles_x, int step, int32_t* order,
                             hipStream_t stream);

} // namespace spd
