// sp_path.hpp -- device implementation of the reference's per-pixel path (gfx950), bit-exact.
//
// One 64-lane wave renders one 8x8 tile (base/Tile.h:10 k_tile_dimension = 8), lane = Morton
// index inside the tile (base/Tile.h TilePixelIterator), exactly the pixel order of
// main.cpp:91.  Waves are persistent: each grabs tiles from an atomic queue until the list is
// drained (the device analogue of TileScheduler::get_next_tile), so a single launch covers the
// frame with no tail of idle CUs.  Each lane runs the reference's sample loop for its pixel
// (main.cpp:94-102): R2 pixel jitter -> PerspectiveCamera ray -> Integrator -> running sum ->
// divide by spp.  The pixel's std::mt19937_64 lives in HBM as two 312-word generations; the
// next generation is twisted ahead of need at wave-synchronous points so lanes rarely twist
// alone.
//
// Numerics: every float operation follows the reference's order; FMAs only where the reference
// issues them (sp_math.h).  Build flags: -ffp-contract=off, IEEE division/sqrt, denormals kept.
#pragma once
#include "sp_device.hpp"

namespace spd {
inline namespace SPD_LAYOUT_NS { // sp_device.hpp: one namespace per RNG state layout

using namespace spm;

// ============================================================================ wave-level profile
// Diagnostic build only (-DSP_WAVE_PROF, tools/gpu_wprof.sh): for each region k the wave's shader
// clocks inside it (slot 2k) and those clocks times the lanes active in it (slot 2k + 1), so the
// region's share of wave time and its lane occupancy come out separately.  Regions:
// 0 = a whole sample (integrate), 1 = the 16-sample glossy rho estimate, 2 = closest-hit queries
// (camera / extension rays: their entry occupancy is the fraction of paths alive), 3 = shadow and
// MIS-ray queries; IterativeRRNEE's merged query pass (mq_run) adds 5 = the whole pass and 4 = its
// walk steps, timed per loop iteration, so 4's occupancy is that of the lanes still walking;
// 6 / 7 = the steps of every 8-wide closest-hit / any-hit walk (per iteration, like 4).
// Written by the first active lane into a per-wave LDS row,
// flushed to the render's tile_diag buffer at kernel end (sp_mega.hpp).
#ifdef SP_WAVE_PROF
static __shared__ unsigned long long wprof_lds[16 * 16];
__device__ __forceinline__ void wprof_end(int k, uint64_t t0)
{
    const uint64_t dt    = __builtin_amdgcn_s_memtime() - t0;
    const uint64_t m     = __ballot(1);
    const int      first = __ffsll((unsigned long long)m) - 1;
    if ((int)(threadIdx.x & 63) == first) {
        const int w = threadIdx.x >> 6;
        wprof_lds[w * 16 + 2 * k] += dt;
        wprof_lds[w * 16 + 2 * k + 1] += dt * (uint64_t)__popcll(m);
    }
}
#define SP_WPROF(k, stmt)                                                                                              \
    do {                                                                                                               \
        const uint64_t t_wp_ = __builtin_amdgcn_s_memtime();                                                           \
        stmt;                                                                                                          \
        wprof_end(k, t_wp_);                                                                                           \
    } while (0)
#else
#define SP_WPROF(k, stmt) stmt
#endif

// ============================================================================ traffic by source
// Diagnostic build only (-DSP_TRAFFIC_DIAG, tools/gpu_traffic_diag.sh): for each source of memory
// requests, the distinct 128-byte lines each wave-level access touches (what the vector L1 asks of
// L2 when it misses) and the bytes the lanes asked for.  Sources: 8-wide BVH nodes, wide-leaf
// triangle records, binary BVH slot records, closest-hit records (indices, normals, material), the
// RNG draws of a lane's own stream, the LDS-DMA touches ahead of a glossy estimate, the words
// another lane's served estimate reads, twists (read + write of a generation) and seeding.  Per
// wave in LDS, flushed to the render's tile_diag buffer (u64 slots 16 + 2k: lines, 17 + 2k: bytes)
// at kernel end (sp_mega.hpp).
#ifdef SP_TRAFFIC_DIAG
enum { TD_NODE, TD_TRI, TD_BIN, TD_HIT, TD_DRAW, TD_TOUCH, TD_SERVED, TD_TWIST, TD_SEED, TD_BOUNCE, TD_N };
static __shared__ unsigned long long tdg_lds[16 * 32];
__device__ __forceinline__ void td_add(int cat, uint64_t lines, uint64_t bytes)
{
    const uint64_t m     = __ballot(1);
    const int      first = __ffsll((unsigned long long)m) - 1;
    if ((int)(threadIdx.x & 63) == first) {
        const int w = threadIdx.x >> 6;
        tdg_lds[w * 32 + 2 * cat] += lines;
        tdg_lds[w * 32 + 2 * cat + 1] += bytes;
    }
}
__device__ __forceinline__ uint32_t td_distinct(uint64_t v, uint64_t todo)
{
    uint32_t cnt = 0;
    while (todo) {
        const int      src = __ffsll((unsigned long long)todo) - 1;
        const uint32_t lo  = (uint32_t)__shfl((int)(uint32_t)v, src, 64);
        const uint32_t hi  = (uint32_t)__shfl((int)(uint32_t)(v >> 32), src, 64);
        todo &= ~__ballot(v == (((uint64_t)hi << 32) | lo));
        ++cnt;
    }
    return cnt;
}
__device__ __forceinline__ void td_lines(int cat, const void* p, int nbytes)
{
    const uint64_t a = (uint64_t)(uintptr_t)p, l0 = a >> 7, l1 = (a + (uint64_t)nbytes - 1) >> 7;
    const uint64_t m = __ballot(1);
    uint32_t cnt = td_distinct(l0, m);
    cnt += td_distinct(l1 != l0 ? l1 : ~0ull, __ballot(l1 != l0));
    td_add(cat, cnt, (uint64_t)__popcll(m) * (uint64_t)nbytes);
}
// a twist by the active lanes: each reads and writes one 312-word generation; with 4-word lane
// blocks a 128-byte line holds 4 lanes' blocks, 78 lines per 4-lane group and direction
__device__ __forceinline__ void td_twist(int cat)
{
    const uint64_t m = __ballot(1);
    uint64_t groups = 0;
    for (int g = 0; g < 16; ++g) groups += ((m >> (4 * g)) & 0xfull) ? 1 : 0;
    td_add(cat, groups * 78 * 2, (uint64_t)__popcll(m) * 312 * 8 * 2);
}
#define SP_TD(stmt) stmt
#else
#define SP_TD(stmt)
#endif

// ============================================================================ per-lane state
// The RSQRTSS table as a kernel holds it (LDS copy, or the global original): t -> the header
// {bits, zero_result, denorm_result, pack_shift, pack_hi} (sp_device.hpp), entries at t + RSQ_HDR.
struct Rsq {
    const uint32_t* t;
};
__device__ __forceinline__ float rsqrt_ref(float a, const Rsq& q)
{
    const uint4    h  = *reinterpret_cast<const uint4*>(q.t);
    const uint32_t hi = q.t[4];
    RsqrtTable     tb{ q.t + RSQ_HDR, (int32_t)h.x, h.y, h.z, (int32_t)h.w, hi };
    return rsqrt_newton(a, rsqrtss_emulated(a, tb));
}
__device__ __forceinline__ f3 normalize(f3 a, const Rsq& q) { return scale(a, rsqrt_ref(dot(a, a), q)); }

// Correctly rounded sqrt of max(0, 1 - v * v)-shaped arguments: x is +0 or at least 2^-24 (1 - v^2
// below 1 is exact near 1 and at least 1 - (1 - 2^-24)), never denormal, negative or inf.  This is
// the compiler's own exact f32 sqrt (v_sqrt_f32 and a one-ulp correction from two FMA residuals)
// without the two parts such x never reach: scaling inputs below 2^-96, and passing 0 / inf
// through (for +0 the correction already returns +0).  16 -> 9 instructions, same bits.
#ifndef SP_SQRT_UNIT
#define SP_SQRT_UNIT 1
#endif
__device__ __forceinline__ float sqrt_unit(float x)
{
#if SP_SQRT_UNIT
    const float s  = __builtin_amdgcn_sqrtf(x);
    const float sd = __uint_as_float(__float_as_uint(s) - 1u);
    const float su = __uint_as_float(__float_as_uint(s) + 1u);
    const float vp = __builtin_fmaf(-sd, s, x);
    const float vs = __builtin_fmaf(-su, s, x);
    float       r  = (vp <= 0.0f) ? sd : s;
    r              = (vs > 0.0f) ? su : r;
    return r;
#else
    return sqrt_f(x);
#endif
}

// Draw-ahead window: the next RNG_PF words of the current generation are loaded RNG_PF draws
// before they are consumed, so a draw does not wait for a global load (the state lives in HBM,
// 160 KB per wave).  The window never crosses into the other buffer and is emptied at every
// buffer switch, so the stream is the same word sequence as without it.
#ifndef SP_RNG_PF
#define SP_RNG_PF 2
#endif
#ifndef SP_XP_SERVED_FREE
#define SP_XP_SERVED_FREE 0
#endif // timing-only bound (SP_XP_* below)
constexpr int RNG_PF = SP_RNG_PF;
struct Rng {
    uint64_t* base;  // this lane's base in its wave slot's state (sp_device.hpp mt_off layout)
    int       cur;   // generation buffer being consumed
    int       idx;   // next word in it
    int       ready; // other buffer already holds the next generation
    uint32_t  draws;
    // Generation store (sp_chunk.hip): with lin, buffer b + 1 follows buffer b (a per-pixel array
    // of successive generations) instead of the two-buffer ring; with pre, every generation is
    // already there, so a buffer switch never twists.
    int       lin = 0, pre = 0;
    int       pfn = 0;        // valid words in pf (words idx .. idx + pfn - 1 of buffer cur)
#ifdef SP_TRAFFIC_DIAG
    int       td_cat = TD_DRAW; // served estimates read another lane's words: TD_SERVED
#endif
    uint64_t  pf[RNG_PF > 0 ? RNG_PF : 1];
#if SP_SERVE_RHO
    // Wave-served selection weights (serve_rho): the estimates of this lane's next eval / pdf /
    // sample call sites were computed by the wave at stream positions srv_pos, + srv_dc and
    // + 2 srv_dc + srv_coat (draw counts); glossy_weights takes them from srv_w when the stream is
    // exactly there.
    // srv_on: 0 off; 1 served weights available (srv_B: eval / pdf / sample of the light being
    // estimated, srv_A: the bounce's own deferred Material::sample, its estimate at srv_posA).
    int       srv_on  = 0;
    bool      srv_A = false, srv_B = false;
    uint32_t  srv_pos = 0, srv_dc = 0, srv_coat = 0, srv_posA = 0, srv_pwA = 0;
#endif
};

__device__ __forceinline__ uint64_t* mt_buf(Rng& r, int b) { return r.base + (size_t)b * MT_GEN_WORDS; }
__device__ __forceinline__ int       mt_next(const Rng& r) { return r.lin ? r.cur + 1 : r.cur ^ 1; }

// B = twist(A) without modifying A (in-place MT19937-64 twist split over two buffers), for twists
// at points where few registers are live (rng_prepare at a sample start, rng_skip).  A and B are
// different generations (__restrict__), and the words are processed in blocks of U words:
// a block's loads are all issued before its first store.  Without that the compiler had to assume
// that a store to B could change A, so every 4-word step waited for its loads to return before
// the next step's loads were issued -- about 80 dependent memory round trips per twist.
// Block sizes, measured (profiles/r02/s6/ab_twist.txt): 12 at rng_prepare (bunny 1080p 2815-2858 ->
// 2949-2955 Mrays/s, elf 554 -> 586; 16 and 24 spill around the sample loop: elf 411 at 24), 24 in
// the chunk pipeline's stream replay (ck_count, few other live values: 8-way shard 2150 -> 2360).
#ifndef SP_TWIST_BLOCK
#define SP_TWIST_BLOCK 12
#endif
#ifndef SP_TWIST_SKIP_BLOCK // 12 since the one-pass twist (2-way shard +0.9 %, 8-way level: profiles/r04/rng_layout/ab_skip_block.txt)
#define SP_TWIST_SKIP_BLOCK 12
#endif
// words k .. k + NW - 1 of B; the words mixed in come from A[k + M] (first part) or B[k - (N - M)]
template <int NW, bool SECOND>
__device__ __forceinline__ void mt_twist_words(const uint64_t* __restrict__ A, uint64_t* __restrict__ B, int k, uint64_t& ak)
{
    if constexpr (NW > 0) {
        uint64_t a1[NW], am[NW];
#pragma unroll
        for (int j = 0; j < NW; ++j) {
            a1[j] = A[mt_off(k + j + 1)];
            am[j] = SECOND ? B[mt_off(k + j - (MT_N - MT_M))] : A[mt_off(k + j + MT_M)];
        }
#pragma unroll
        for (int j = 0; j < NW; ++j) {
            B[mt_off(k + j)] = am[j] ^ mt_mix(ak, a1[j]);
            ak              = a1[j];
        }
    }
}
struct MtOff {
    __device__ __forceinline__ size_t operator()(int k) const { return mt_off(k); }
};
// SP_TWIST_FUSED: the one-pass forms of sp_twist4.h (every word of A loaded once, B not read back)
#ifndef SP_TWIST_FUSED
#define SP_TWIST_FUSED 1
#endif
template <int U>
__device__ __forceinline__ void mt_twist_blocked(const uint64_t* __restrict__ A, uint64_t* __restrict__ B)
{
#ifndef SP_TWIST_GROUPED
#define SP_TWIST_GROUPED 1
#endif
    if constexpr (MT_BLK == 4 && SP_TWIST_GROUPED) { // 4-word lane groups, 3 per block (sp_twist4.h)
        if (SP_TWIST_FUSED) mt_twist_grouped4_fused<3>(A, B);
        else mt_twist_grouped4<3>(A, B);
        return;
    }
    if constexpr (SP_TWIST_FUSED) {
        mt_twist_fused<U>(A, B, MtOff{});
        return;
    }
    constexpr int H  = MT_N - MT_M;     // words 0 .. H - 1 mix with A[k + M]
    constexpr int N2 = MT_N - 1 - H;    // words H .. N - 2 mix with B[k - H]
    uint64_t      ak = A[0];
#pragma unroll 1
    for (int b = 0; b < H / U; ++b) mt_twist_words<U, false>(A, B, b * U, ak);
    mt_twist_words<H % U, false>(A, B, (H / U) * U, ak);
#pragma unroll 1
    for (int b = 0; b < N2 / U; ++b) mt_twist_words<U, true>(A, B, H + b * U, ak);
    mt_twist_words<N2 % U, true>(A, B, H + (N2 / U) * U, ak);
    B[mt_off(MT_N - 1)] = B[mt_off(MT_M - 1)] ^ mt_mix(ak, B[0]);
}

// B = twist(A) without modifying A: the compact form, for twists inside register-heavy code (the
// in-draw fallback, rng_reserve), where the blocked form's 4 x SP_TWIST_BLOCK live registers would
// spill.
#ifndef SP_TWIST_INTO_FUSED
#define SP_TWIST_INTO_FUSED 0
#endif
__device__ __forceinline__ void mt_twist_into(const uint64_t* A, uint64_t* B)
{
    if constexpr (SP_TWIST_INTO_FUSED > 0) { // one pass, SP_TWIST_INTO_FUSED words per block of loads
        mt_twist_fused<SP_TWIST_INTO_FUSED>(A, B, MtOff{});
        return;
    }
    uint64_t ak = A[0];
#pragma unroll 4
    for (int k = 0; k < MT_N - MT_M; ++k) {
        const uint64_t ak1 = A[mt_off(k + 1)];
        B[mt_off(k)]       = A[mt_off(k + MT_M)] ^ mt_mix(ak, ak1);
        ak                 = ak1;
    }
#pragma unroll 4
    for (int k = MT_N - MT_M; k < MT_N - 1; ++k) {
        const uint64_t ak1 = A[mt_off(k + 1)];
        B[mt_off(k)]       = B[mt_off(k - (MT_N - MT_M))] ^ mt_mix(ak, ak1);
        ak                 = ak1;
    }
    B[mt_off(MT_N - 1)] = B[mt_off(MT_M - 1)] ^ mt_mix(ak, B[0]);
}

__device__ __forceinline__ void rng_seed(Rng& r, uint32_t seed)
{
    uint64_t* b = mt_buf(r, 0);
    uint64_t  x = (uint64_t)seed;
    b[0]        = x;
    for (int i = 1; i < MT_N; ++i) {
        x          = mt_seed_next(x, (uint64_t)i);
        b[mt_off(i)] = x;
    }
    r.cur   = 0;
    r.idx   = MT_N; // std::mt19937_64 starts with _M_p = n: first draw twists
    r.ready = 0;
    r.draws = 0;
    r.pfn   = 0;
}

// rng_seed followed by the first twist, without storing or re-reading the seeded state: the engine
// starts with _M_p = n, so the seeded words are only ever read by that twist.  Generation 1 goes
// straight into the next buffer: word k < M mixes seeded words k, k + 1 and k + M, taken from two
// running seed chains (the second started M steps ahead); word k in [M, N - 1) mixes seeded words
// k, k + 1 with the new word k - M, written M words before (read back in blocks of 12, all loads of
// a block issued before its stores).  The same state as rng_seed + mt_twist_blocked (cur = 0 at
// its end, next buffer ready).
#ifndef SP_SEED_FUSED
#define SP_SEED_FUSED 1
#endif
__device__ __forceinline__ void rng_seed_twisted(Rng& r, uint32_t seed)
{
    static_assert(MT_N - MT_M == MT_M, "two seed chains M apart cover words 0 .. N - 1");
    SP_TD(td_twist(TD_SEED)); // writes a generation, reads back part of it (counted as a twist's)
    r.cur         = 0;
    uint64_t*  B  = mt_buf(r, mt_next(r));
    uint64_t   xk = (uint64_t)seed, xm = (uint64_t)seed;
#pragma unroll 4
    for (int i = 1; i <= MT_M; ++i) xm = mt_seed_next(xm, (uint64_t)i);
    uint64_t b0 = 0;
#pragma unroll 4
    for (int k = 0; k < MT_M; ++k) {
        const uint64_t xk1 = mt_seed_next(xk, (uint64_t)(k + 1));
        const uint64_t w   = xm ^ mt_mix(xk, xk1);
        B[mt_off(k)]       = w;
        if (k == 0) b0 = w;
        xm = mt_seed_next(xm, (uint64_t)(k + MT_M + 1));
        xk = xk1;
    }
    constexpr int U = 12, NW = MT_N - 1 - MT_M; // words M .. N - 2
#pragma unroll 1
    for (int k0 = MT_M; k0 < MT_M + NW; k0 += U) {
        uint64_t p[U];
#pragma unroll
        for (int j = 0; j < U; ++j)
            if (k0 + j < MT_M + NW) p[j] = B[mt_off(k0 + j - MT_M)];
#pragma unroll
        for (int j = 0; j < U; ++j)
            if (k0 + j < MT_M + NW) {
                const uint64_t xk1 = mt_seed_next(xk, (uint64_t)(k0 + j + 1));
                B[mt_off(k0 + j)]  = p[j] ^ mt_mix(xk, xk1);
                xk                 = xk1;
            }
    }
    B[mt_off(MT_N - 1)] = B[mt_off(MT_M - 1)] ^ mt_mix(xk, b0);
    r.idx   = MT_N;
    r.ready = 1;
    r.draws = 0;
    r.pfn   = 0;
}

// Twist ahead at a wave-synchronous point (sample / bounce start).  A lane may compute its next
// generation any time after starting the current one, so all lanes whose next buffer is stale
// twist together -- but only once some lane is within RNG_MARGIN draws of exhausting its buffer.
// Twists are thus batched (about one per 312 draws per wave instead of one per sample), and the
// in-draw fallback (rng_raw) keeps the stream exact when a path draws more than the margin.
#ifndef SP_RNG_MARGIN
#define SP_RNG_MARGIN 96
#endif
constexpr int RNG_MARGIN = SP_RNG_MARGIN;
__device__ __forceinline__ void rng_prepare(Rng& r)
{
    const bool urgent = !r.ready && r.idx >= MT_N - RNG_MARGIN;
    if (__any(urgent)) {
        if (!r.ready) {
            SP_TD(td_twist(TD_TWIST));
            mt_twist_blocked<SP_TWIST_BLOCK>(mt_buf(r, r.cur), mt_buf(r, mt_next(r)));
            r.ready = 1;
        }
    }
}

// NT ("no twist"): the caller has made sure the next generation is ready (rng_reserve), so the
// twist is not inlined at this draw -- its code and registers stay out of hot loops.
template <bool NT = false>
__device__ __forceinline__ uint64_t rng_raw(Rng& r)
{
    if (r.idx >= MT_N) {
        if (!NT && !r.ready) {
            SP_TD(td_twist(TD_TWIST));
            mt_twist_into(mt_buf(r, r.cur), mt_buf(r, mt_next(r)));
        }
        r.cur   = mt_next(r);
        r.idx   = 0;
        r.ready = r.pre;
        r.pfn   = 0;
    }
    const uint64_t* b = mt_buf(r, r.cur);
    uint64_t        w;
    if (RNG_PF > 0 && r.pfn > 0) {
        w = r.pf[0];
#pragma unroll
        for (int k = 0; k + 1 < RNG_PF; ++k) r.pf[k] = r.pf[k + 1];
        --r.pfn;
    } else if (SP_XP_SERVED_FREE && r.lin == 2) { // timing-only bound: hashed words, no read
        w = ((uint64_t)(r.idx + 1000 * r.cur + 7) * 0x9E3779B97F4A7C15ull) ^ (uint64_t)(uintptr_t)r.base;
    } else {
        SP_TD(td_lines(r.td_cat, &b[mt_off(r.idx)], 8));
        w = b[mt_off(r.idx)];
    }
    ++r.idx;
    // top the window up to RNG_PF words ahead (static indices: the window stays in registers)
#pragma unroll
    for (int k = 0; k < RNG_PF; ++k)
        if (r.pfn == k && r.idx + k < MT_N) {
            SP_TD(td_lines(r.td_cat, &b[mt_off(r.idx + k)], 8));
            r.pf[k] = b[mt_off(r.idx + k)];
            r.pfn   = k + 1;
        }
    ++r.draws;
    return mt_temper(w);
}

// Advance the stream by n draws without reading them: the same state (buffers, position,
// twists) as n rng_raw calls.  Used where only the count of a span of draws is known.
__device__ __forceinline__ void rng_skip(Rng& r, int n)
{
    while (n > 0) {
        if (r.idx >= MT_N) {
            if (!r.ready) {
                SP_TD(td_twist(TD_TWIST));
                mt_twist_blocked<SP_TWIST_SKIP_BLOCK>(mt_buf(r, r.cur), mt_buf(r, mt_next(r)));
            }
            r.cur   = mt_next(r);
            r.idx   = 0;
            r.ready = r.pre;
        }
        const int take = (n < MT_N - r.idx) ? n : MT_N - r.idx;
        r.idx += take;
        r.draws += (uint32_t)take;
        n -= take;
    }
    r.pfn = 0;
}

// rng_skip for n words that rng_reserve(n) has made twist-free (n <= MT_N): the same state,
// without inlining a twist at the call site.
__device__ __forceinline__ void rng_skip_reserved(Rng& r, int n)
{
    const int t = r.idx + n;
    if (t > MT_N) {
        r.cur   = mt_next(r);
        r.idx   = t - MT_N;
        r.ready = r.pre;
    } else {
        r.idx = t;
    }
    r.draws += (uint32_t)n;
    r.pfn = 0;
}

// Pull the next n words of this lane's stream toward the CU before they are drawn.  The state
// (2.5 KB per pixel, gigabytes per frame) was written many kernels ago and lives in HBM, so each
// draw of a 32-draw glossy estimate would otherwise wait one full memory latency.  The words are
// fetched with LDS-DMA loads into a sink that nobody reads: no VGPR is held, all n are in flight
// at once, and the draws that follow hit L2.  Only the cache state changes -- the stream, the
// buffers and every value drawn are exactly as without it.  Rows past the current generation are
// touched in the next buffer only when it already holds the next generation.
__device__ __forceinline__ void rng_touch(const Rng& r, int n, __attribute__((address_space(3))) void* sink)
{
    if (SP_XP_SERVED_FREE && r.lin == 2) return;
    const uint64_t* cur  = r.base + (size_t)r.cur * MT_GEN_WORDS;
    const uint64_t* next = r.base + (size_t)mt_next(r) * MT_GEN_WORDS;
    if constexpr (MT_BLK == 1) {
#pragma unroll 4
        for (int k = 0; k < n; ++k) {
            const int row = r.idx + k;
            if (row < MT_N) __builtin_amdgcn_global_load_lds((const void*)(cur + mt_off(row)), sink, 4, 0, 0);
            else if (r.ready) __builtin_amdgcn_global_load_lds((const void*)(next + mt_off(row - MT_N)), sink, 4, 0, 0);
        }
    } else { // one touch per line: words idx .. idx + n - 1 of this generation, the rest of the next
        const int end = r.idx + n;
        for (int row = r.idx; row < end && row < MT_N; row = (row / MT_BLK + 1) * MT_BLK) {
            SP_TD(td_lines(TD_TOUCH, cur + mt_off(row), 4));
            __builtin_amdgcn_global_load_lds((const void*)(cur + mt_off(row)), sink, 4, 0, 0);
        }
        if (r.ready)
            for (int row = 0; row < end - MT_N; row += MT_BLK) {
                SP_TD(td_lines(TD_TOUCH, next + mt_off(row), 4));
                __builtin_amdgcn_global_load_lds((const void*)(next + mt_off(row)), sink, 4, 0, 0);
            }
    }
}

// Make the next n draws twist-free: if they run past the current generation and the next one is
// not there yet, twist it now.  A twist reads only the current generation, so computing it before
// its first word is drawn gives the same words as twisting at the boundary.
__device__ __forceinline__ void rng_reserve(Rng& r, int n)
{
    if (!r.ready && r.idx + n > MT_N) {
        SP_TD(td_twist(TD_TWIST));
        mt_twist_into(mt_buf(r, r.cur), mt_buf(r, mt_next(r)));
        r.ready = 1;
    }
}

// SP_RHO_TOUCH: the 16-sample glossy estimate touches its 32 words first; the DMA target is one
// 256-byte LDS sink per block.  Per translation unit: on in the DirectLighting megakernel (with
// no draw-ahead window: bunny 2720 -> 2762 Mrays/s, profiles/r02/s5), the sample chunks (round 2
// session 6) and the IterativeRRNEE megakernel once its estimates are served across the wave
// (739-745 -> 746-757 on elf; the lock-step kernel had lost with it, 553 -> 541).
#ifndef SP_RHO_TOUCH
#define SP_RHO_TOUCH 0
#endif
#if SP_RHO_TOUCH
static __shared__ uint32_t rho_rng_sink[64];
#endif

// Two consecutive draws.  With lane blocks of 4 words (MT_BLK >= 2) words 2j and 2j + 1 of a
// generation are one aligned 16-byte pair, so two draws that start at an even position are one
// dwordx4 load instead of two dwordx2 loads: half the wave-level RNG loads -- and half the
// vector-L1 tag lookups -- where lanes read scattered streams (a served estimate reads 32 words of
// ANOTHER lane's stream: per wave instruction up to 64 lines, the largest source of lookups in the
// elf frame).  Same words in the same order (a generation has an even number of
// words, so a pair never straddles two); at an odd position the draws are taken one by one.
// Per translation unit: on in the DirectLighting megakernel (bunny 1080p @ 256 spp +0.2-0.5 %,
// spheres 1024^2 @ 64 spp +1-3 %), off in IterativeRRNEE's (elf 1024^2 @ 16 spp 1028-1031 ->
// 993-998, its 8-way shard 1220-1224 -> 1174-1179 Mrays/s; profiles/r05/rng_pair/).
#ifndef SP_RNG_PAIR
#define SP_RNG_PAIR 0
#endif
// PAIR: the pair form for this call (default SP_RNG_PAIR; IterativeRRNEE's served estimates choose
// their own, SP_SERVED_PAIR).
#ifndef SP_SERVED_PAIR
#define SP_SERVED_PAIR SP_RNG_PAIR
#endif
#ifndef SP_SERVED_ALIGNED
#define SP_SERVED_ALIGNED SP_RHO_ALIGNED
#endif
#ifndef SP_SERVED_TOUCH
#define SP_SERVED_TOUCH SP_RHO_TOUCH
#endif
template <bool NT = false, bool PAIR = (SP_RNG_PAIR != 0)>
__device__ __forceinline__ void rng_raw2(Rng& r, uint64_t& w0, uint64_t& w1)
{
    // pairs need even lane blocks: with MT_BLK % 2 != 0 (e.g. 3) words 2j, 2j + 1 can sit in two
    // blocks and a lane's block is not 16-byte aligned
    static_assert(!PAIR || MT_BLK == 1 || MT_BLK % 2 == 0, "SP_RNG_PAIR needs an even MT_BLK");
    if constexpr (PAIR && MT_BLK >= 2 && MT_BLK % 2 == 0 && RNG_PF == 0) {
        if (r.idx >= MT_N) { // the buffer switch of rng_raw
            if (!NT && !r.ready) {
                SP_TD(td_twist(TD_TWIST));
                mt_twist_into(mt_buf(r, r.cur), mt_buf(r, mt_next(r)));
            }
            r.cur   = mt_next(r);
            r.idx   = 0;
            r.ready = r.pre;
            r.pfn   = 0;
        }
        if ((r.idx & 1) == 0) {
            const uint64_t* b = mt_buf(r, r.cur) + mt_off(r.idx);
            SP_TD(td_lines(r.td_cat, b, 16));
            const ulonglong2 p = *reinterpret_cast<const ulonglong2*>(b);
            w0 = mt_temper(p.x);
            w1 = mt_temper(p.y);
            r.idx += 2;
            r.draws += 2;
            return;
        }
    }
    w0 = rng_raw<NT>(r);
    w1 = rng_raw<NT>(r);
}

// IncoherentSampler::get_next_1D / get_next_2D (math/Sampler.h:110-118)
template <bool NT = false>
__device__ __forceinline__ float next1D(Rng& r) { return canonical_from_u64(rng_raw<NT>(r)); }
struct P2 {
    float x, y;
};
__device__ __forceinline__ P2 next2D(Rng& r)
{
    uint64_t a, b;
    rng_raw2(r, a, b);
    P2 p;
    p.x = canonical_from_u64(a); // braced-init-list: left-to-right
    p.y = canonical_from_u64(b);
    return p;
}

// ============================================================================ rays & hits
struct Ray {
    f3 o, d;
};
__device__ __forceinline__ f3 ray_at(const Ray& r, float t) { return add(r.o, scale(r.d, t)); } // math/Ray.h:180

// math/Ray.h:201
__device__ __forceinline__ float ray_offset(float cos_d) { return (cos_d == 0.0f) ? k_ray_epsilon : k_ray_epsilon / cos_d; }
__device__ __forceinline__ float ray_offset(f3 n, f3 d) { return ray_offset(abs_f(dot(n, d))); }

// math/BBox.h:254 intersect_p(BBox, Ray, RayLimits)
__device__ __forceinline__ bool box_hit(const Node& n, const Ray& r, const f3& inv, float tmin, float tmax)
{
    float t0 = tmin, t1 = tmax;
    {
        float tn = (n.lo[0] - r.o.x) * inv.x, tf = (n.hi[0] - r.o.x) * inv.x;
        if (tn > tf) { const float s = tn; tn = tf; tf = s; }
        t0 = std_max(tn, t0);
        t1 = std_min(tf, t1);
        if (t0 > t1) return false;
    }
    {
        float tn = (n.lo[1] - r.o.y) * inv.y, tf = (n.hi[1] - r.o.y) * inv.y;
        if (tn > tf) { const float s = tn; tn = tf; tf = s; }
        t0 = std_max(tn, t0);
        t1 = std_min(tf, t1);
        if (t0 > t1) return false;
    }
    {
        float tn = (n.lo[2] - r.o.z) * inv.z, tf = (n.hi[2] - r.o.z) * inv.z;
        if (tn > tf) { const float s = tn; tn = tf; tf = s; }
        t0 = std_max(tn, t0);
        t1 = std_min(tf, t1);
        if (t0 > t1) return false;
    }
    return true;
}

// shapes/Triangle.h:97 intersect_impl -- returns t, beta, gamma
__device__ __forceinline__ bool tri_hit(const float4& q0, const float4& q1, const float4& q2, const Ray& ray, float tmin,
                                        float tmax, float& t_out, float& beta_out, float& gamma_out)
{
    const float A = q0.x - q1.x, B = q0.y - q1.y, C = q0.z - q1.z;
    const float D = q0.x - q2.x, E = q0.y - q2.y, F = q0.z - q2.z;
    const float G = ray.d.x, H = ray.d.y, I = ray.d.z;
    const float J = q0.x - ray.o.x, K = q0.y - ray.o.y, L = q0.z - ray.o.z;
    const float EIHF  = fma_f(E, I, -(H * F));
    const float GFDI  = fma_f(G, F, -(D * I));
    const float DHEG  = fma_f(D, H, -(E * G));
    const float denom = fma_f(A, EIHF, fma_f(B, GFDI, C * DHEG));
    if (denom == 0) return false;
    const float beta = fma_f(J, EIHF, fma_f(K, GFDI, L * DHEG)) / denom;
    if (beta <= 0.0f || beta >= 1.0f) return false;
    const float AKJB  = fma_f(A, K, -(J * B));
    const float JCAL  = fma_f(J, C, -(A * L));
    const float BLKC  = fma_f(B, L, -(K * C));
    const float gamma = fma_f(I, AKJB, fma_f(H, JCAL, G * BLKC)) / denom;
    if (gamma <= 0.0f || beta + gamma >= 1.0f) return false;
    const float t = -fma_f(F, AKJB, fma_f(E, JCAL, D * BLKC)) / denom;
    if (t < tmin || t > tmax) return false;
    t_out     = t;
    beta_out  = beta;
    gamma_out = gamma;
    return true;
}

// shapes/Sphere.h:295 intersect_impl (t only; normal derived at the end)
__device__ __forceinline__ bool sphere_t(const aff& w2o, const Ray& ray, float tmin, float tmax, float& t_out)
{
    const f3    o    = xfm_point(w2o, ray.o);
    const f3    d    = xfm_vector(w2o, ray.d);
    const float a    = dot(d, d);
    const float b    = 2.0f * dot(d, o);
    const float c    = dot(o, o) - 1.0f * 1.0f;
    float       disc = b * b - 4.0f * a * c;
    if (disc > 0.0f) {
        disc    = sqrt_f(disc);
        float t = (-b - disc) / (2.0f * a);
        if (t < tmin) t = (-b + disc) / (2.0f * a);
        if (t < tmin || t > tmax) return false;
        t_out = t;
        return true;
    }
    return false;
}

// shapes/Plane.h:391 intersect_impl (t only)
__device__ __forceinline__ bool plane_t(const aff& w2o, const Ray& ray, float tmin, float tmax, float& t_out)
{
    const f3 d = xfm_vector(w2o, ray.d);
    if (d.y == 0.0f) return false;
    const f3    o = xfm_point(w2o, ray.o);
    const float t = -o.y / d.y;
    if (t < tmin || t > tmax) return false;
    t_out = t;
    return true;
}

struct Hit {
    float    t;
    uint32_t code; // kind << 30 | index ; 0xffffffff = none
    float    beta, gamma;
    uint32_t slot = 0xffffffffu; // 8-wide walks: wide slot of the hit primitive (none / unbounded: ~0)
};

constexpr uint32_t KIND_TRI = 0u, KIND_SPHERE = 1u, KIND_PLANE = 2u;

struct Isect {
    float t;
    f3    n, p;
    int   material;
};

// Shape-specific surface data for the final closest hit (identical arithmetic to the reference,
// which computes it for every accepted candidate).
__device__ __forceinline__ Isect finish_hit(const Scene& sc, const Hit& h, const Ray& ray, const Rsq& q)
{
    Isect          is;
    const uint32_t kind = h.code >> CODE_SHIFT;
    const uint32_t id   = h.code & CODE_MASK;
    is.t = h.t;
    is.p = ray_at(ray, h.t);
    if (kind == KIND_TRI) {
        SP_TD(td_lines(TD_HIT, &sc.indices[3 * id], 12));
        SP_TD(td_lines(TD_HIT, &sc.tri_material[id], 4));
        const uint32_t i0 = sc.indices[3 * id], i1 = sc.indices[3 * id + 1], i2 = sc.indices[3 * id + 2];
        SP_TD(td_lines(TD_HIT, &sc.normals[3 * i0], 12));
        SP_TD(td_lines(TD_HIT, &sc.normals[3 * i1], 12));
        SP_TD(td_lines(TD_HIT, &sc.normals[3 * i2], 12));
        const f3 n0 = mk(sc.normals[3 * i0], sc.normals[3 * i0 + 1], sc.normals[3 * i0 + 2]);
        const f3 n1 = mk(sc.normals[3 * i1], sc.normals[3 * i1 + 1], sc.normals[3 * i1 + 2]);
        const f3 n2 = mk(sc.normals[3 * i2], sc.normals[3 * i2 + 1], sc.normals[3 * i2 + 2]);
        const float alpha = 1.0f - h.beta - h.gamma;
        is.n        = normalize(madd(alpha, n0, madd(h.beta, n1, scale(h.gamma, n2))), q);
        is.material = sc.tri_material[id];
    } else if (kind == KIND_SPHERE) {
        const Shape& s = sc.shapes[id];
        const f3     o = xfm_point(s.w2o, ray.o);
        const f3     d = xfm_vector(s.w2o, ray.d);
        const f3     nl = divs(madd(h.t, d, o), 1.0f);
        is.n        = normalize(xfm_vector(s.nrm, nl), q);
        is.material = s.material;
    } else {
        const Shape& s = sc.shapes[id];
        is.n        = xfm_vector(s.nrm, mk(0.0f, 1.0f, 0.0f));
        is.material = s.material;
    }
    return is;
}

// ---------------------------------------------------------------- timing-only bounds (SP_XP_*)
// Experiment builds only (wrong or unchanged images, never the product): each measures how much a
// cost could matter before anything is built against it.
//   SP_XP_DUP 1: every 8-wide node fetch is issued twice (the second through an address the
//     compiler cannot prove equal, its words OR-ed in under a zero mask): twice the vector-L1
//     lookups of node fetches, same walk and same image -- the sensitivity of the frame to them;
//     2: the wide-leaf triangle records too.
//   SP_XP_FASTLIBM: expf / logf / powf / sinf / cosf as the native f32 instructions (wrong image):
//     the upper bound of replacing the exact glibc emulation's f64 arithmetic.
//   SP_XP_SERVED_FREE: served estimates (IterativeRRNEE) draw hashed words instead of reading the
//     owner's stream (wrong image): the upper bound of making their reads free.
#ifndef SP_XP_DUP
#define SP_XP_DUP 0
#endif
#if SP_XP_DUP
__device__ __forceinline__ uint32_t xp_zero()
{
    uint32_t z;
    asm volatile("v_mov_b32 %0, 0" : "=v"(z));
    return z;
}
__device__ __forceinline__ void xp_or(uint4& w, const uint4& d, uint32_t z)
{
    w.x |= d.x & z; w.y |= d.y & z; w.z |= d.z & z; w.w |= d.w & z;
}
__device__ __forceinline__ void xp_dup(const uint4* p, uint4& w0, uint4& w1, uint4& w2, uint4& w3, uint4& w4)
{
    const uint32_t z = xp_zero();
    const uint4*   q = p + z;
    const uint4    d0 = q[0], d1 = q[1], d2 = q[2], d3 = q[3], d4 = q[4];
    xp_or(w0, d0, z); xp_or(w1, d1, z); xp_or(w2, d2, z); xp_or(w3, d3, z); xp_or(w4, d4, z);
}
__device__ __forceinline__ void xp_orf(float4& w, const float4& d, uint32_t z)
{
    w.x = __uint_as_float(__float_as_uint(w.x) | (__float_as_uint(d.x) & z));
    w.y = __uint_as_float(__float_as_uint(w.y) | (__float_as_uint(d.y) & z));
    w.z = __uint_as_float(__float_as_uint(w.z) | (__float_as_uint(d.z) & z));
    w.w = __uint_as_float(__float_as_uint(w.w) | (__float_as_uint(d.w) & z));
}
__device__ __forceinline__ void xp_dup3(const float4* p, float4& q0, float4& q1, float4& q2)
{
    const uint32_t z = xp_zero();
    const float4*  q = p + z;
    const float4   d0 = q[0], d1 = q[1], d2 = q[2];
    xp_orf(q0, d0, z); xp_orf(q1, d1, z); xp_orf(q2, d2, z);
}
#endif

// Test one primitive code against the ray (closest-hit semantics: t <= tmax accepted).
__device__ __forceinline__ bool prim_closest(const Scene& sc, uint32_t slot, const Ray& ray, float tmin, Hit& h,
                                             const float4* tris = nullptr)
{
    const float4*  st   = tris ? tris : sc.slot_tri;
    const float4   q0   = st[3 * slot]; // p0 | code
    const float4   q1 = st[3 * slot + 1], q2 = st[3 * slot + 2]; // with q0: one memory latency (SP_TRI_EAGER)
    const uint32_t code = __float_as_uint(q0.w);
    const uint32_t kind = code >> CODE_SHIFT;
    if (kind == KIND_TRI) {
        float t, be, ga;
        if (tri_hit(q0, q1, q2, ray, tmin, h.t, t, be, ga)) {
            h.t = t; h.code = code; h.beta = be; h.gamma = ga;
            return true;
        }
        return false;
    }
    const Shape& s = sc.shapes[code & CODE_MASK];
    float        t;
    const bool   hit = (kind == KIND_SPHERE) ? sphere_t(s.w2o, ray, tmin, h.t, t) : plane_t(s.w2o, ray, tmin, h.t, t);
    if (hit) { h.t = t; h.code = code; }
    return hit;
}

// Closest hit on the 8-wide BVH: (t, wide slot) is minimised lexicographically over every primitive
// the ray hits in [tmin, t_max], so the result does not depend on the order a walk meets them --
// the walks that several lanes share (mq_run) and the per-lane walk give the same hit.  (On the SAH
// BVH only equal-t ties are affected, which the reference-order BVH keeps in the reference's
// order: the binary walks use prim_closest.)  A BVH primitive at the unbounded shapes' t wins, as
// with prim_closest (their slot is ~0).
__device__ __forceinline__ bool prim_closest_w(const Scene& sc, uint32_t slot, const Ray& ray, float tmin, Hit& h)
{
    SP_TD(td_lines(TD_TRI, &sc.wslot_tri[3 * slot], 48));
#if SP_XP_DUP >= 2
    float4 q0 = sc.wslot_tri[3 * slot], q1 = sc.wslot_tri[3 * slot + 1], q2 = sc.wslot_tri[3 * slot + 2];
    xp_dup3(&sc.wslot_tri[3 * slot], q0, q1, q2);
#else
    const float4   q0   = sc.wslot_tri[3 * slot]; // p0 | code
    const float4   q1 = sc.wslot_tri[3 * slot + 1], q2 = sc.wslot_tri[3 * slot + 2]; // issued with q0
#endif
    const uint32_t code = __float_as_uint(q0.w);
    const uint32_t kind = code >> CODE_SHIFT;
    float          t, be = 0.0f, ga = 0.0f;
    bool           hit;
    if (kind == KIND_TRI) {
        hit = tri_hit(q0, q1, q2, ray, tmin, h.t, t, be, ga);
    } else {
        const Shape& s = sc.shapes[code & CODE_MASK];
        hit = (kind == KIND_SPHERE) ? sphere_t(s.w2o, ray, tmin, h.t, t) : plane_t(s.w2o, ray, tmin, h.t, t);
    }
    if (!hit || !(t < h.t || slot < h.slot)) return false;
    h.t = t; h.code = code; h.beta = be; h.gamma = ga; h.slot = slot;
    return true;
}

__device__ __forceinline__ bool prim_any(const Scene& sc, uint32_t slot, const Ray& ray, float tmin, float tmax,
                                         const float4* tris = nullptr)
{
    const float4*  st   = tris ? tris : sc.slot_tri;
    SP_TD(td_lines(tris ? TD_TRI : TD_BIN, &st[3 * slot], 48));
#if SP_XP_DUP >= 2
    float4 q0 = st[3 * slot], q1 = st[3 * slot + 1], q2 = st[3 * slot + 2];
    xp_dup3(&st[3 * slot], q0, q1, q2);
#else
    const float4   q0   = st[3 * slot]; // p0 | code
    const float4   q1 = st[3 * slot + 1], q2 = st[3 * slot + 2]; // issued with q0
#endif
    const uint32_t code = __float_as_uint(q0.w);
    const uint32_t kind = code >> CODE_SHIFT;
    if (kind == KIND_TRI) {
        float t, be, ga;
        return tri_hit(q0, q1, q2, ray, tmin, tmax, t, be, ga);
    }
    const Shape& s = sc.shapes[code & CODE_MASK];
    float        t;
    return (kind == KIND_SPHERE) ? sphere_t(s.w2o, ray, tmin, tmax, t) : plane_t(s.w2o, ray, tmin, tmax, t);
}

// LDS traversal stack: entry e of lane l at stack[e * 64 + l].  Entries are nodes whose box
// test is still pending, popped child-0-first: the visiting order of the reference's recursion
// (shapes/BVHAccelerator.h:62-77) with each box tested against the limits current at that time.
struct Stack {
    uint32_t* s;
    int       lane;
    int       depth; // entries; pair traversal keeps each entry's entry distance at s[(e + depth) * 64 + lane]
};

// SAH nodes carry their split axis: the child on the far side of the ray's direction is
// deferred.  Only the visiting order changes (closest hit: equal-distance ties may resolve to
// another primitive; any hit: no change), so the reference-order BVH never uses it.

// Depth-first walk of a binary BVH in the reference's recursion order: a node's second child is
// deferred while the first child's subtree is walked, and box-tested (against the limits current
// then) when the walk comes back to it.  The deferred children live on the LDS stack, or -- for
// BVHs deeper than the LDS budget (Scene::stackless) -- are found again by climbing parent links
// from the finished subtree to the first ancestor entered through its first child: the same
// nodes, in the same order, with the same box tests, and no per-lane memory at all (a degenerate
// median-split tree can nest thousands of levels, like the reference's recursion).
// SL (stackless) is a template parameter so the stack walk compiles to exactly the loop it was.
template <bool SL>
struct BinWalk {
    Stack           st;
    int             sp;
    const Node*     nodes;
    const uint32_t* parents; // SL: parent links
    bool            ordered; // SAH near-first order
    uint32_t        dneg;    // bit a: ray direction component a < 0 (near_is_second without selects)
};
__device__ __forceinline__ uint32_t dir_sign_bits(const f3& d)
{
    return (d.x < 0.0f ? 1u : 0u) | (d.y < 0.0f ? 2u : 0u) | (d.z < 0.0f ? 4u : 0u);
}
template <bool SL>
__device__ __forceinline__ BinWalk<SL> bin_walk(Stack st, const Node* nodes, const uint32_t* parents, bool ordered,
                                                const f3& d)
{
    return BinWalk<SL>{ st, 0, nodes, parents, ordered, dir_sign_bits(d) };
}
template <bool SL>
__device__ __forceinline__ void children_in_order(const BinWalk<SL>& w, const Node& n, const f3&, uint32_t& first,
                                                  uint32_t& second)
{
    first  = n.a & CHILD_MASK;
    second = n.b;
    if (w.ordered && ((w.dneg >> (n.a >> AXIS_SHIFT)) & 1u)) { const uint32_t t = first; first = second; second = t; }
}
template <bool SL>
__device__ __forceinline__ void walk_defer(BinWalk<SL>& w, uint32_t second)
{
    if (SL) return;
    w.st.s[w.sp * 64 + w.st.lane] = second;
    ++w.sp;
}
// The next deferred node after the subtree at `cur` is finished; false when the walk is done.
template <bool SL>
__device__ __forceinline__ bool walk_next(BinWalk<SL>& w, const f3& d, uint32_t& cur)
{
    if (!SL) {
        if (w.sp == 0) return false;
        --w.sp;
        cur = w.st.s[w.sp * 64 + w.st.lane];
        return true;
    }
    while (cur != 0) {
        const uint32_t p = w.parents[cur];
        uint32_t       first, second;
        children_in_order(w, w.nodes[p], d, first, second);
        if (cur == first) {
            cur = second;
            return true;
        }
        cur = p;
    }
    return false;
}


// Slab test of one box with its entry distance (math/BBox.h:254 operation order).
__device__ __forceinline__ bool slab_box(float lx, float ly, float lz, float hx, float hy, float hz, const Ray& r,
                                         const f3& inv, float tmin, float tmax, float& t0_out)
{
    float t0 = tmin, t1 = tmax; // same operation order as box_hit (math/BBox.h:254)
    {
        float tn = (lx - r.o.x) * inv.x, tf = (hx - r.o.x) * inv.x;
        if (tn > tf) { const float s = tn; tn = tf; tf = s; }
        t0 = std_max(tn, t0);
        t1 = std_min(tf, t1);
        if (t0 > t1) return false;
    }
    {
        float tn = (ly - r.o.y) * inv.y, tf = (hy - r.o.y) * inv.y;
        if (tn > tf) { const float s = tn; tn = tf; tf = s; }
        t0 = std_max(tn, t0);
        t1 = std_min(tf, t1);
        if (t0 > t1) return false;
    }
    {
        float tn = (lz - r.o.z) * inv.z, tf = (hz - r.o.z) * inv.z;
        if (tn > tf) { const float s = tn; tn = tf; tf = s; }
        t0 = std_max(tn, t0);
        t1 = std_min(tf, t1);
        if (t0 > t1) return false;
    }
    t0_out = t0;
    return true;
}

// ------------------------------------------------------------------------------ 8-wide BVH
// One 80-byte fetch (5 x dwordx4) tests the boxes of up to 8 children, so a ray's chain of
// dependent node fetches is about a third of the binary walk's.  Child boxes decode to
// supersets of the exact boxes (outward rounding, sp_bvh.cpp build_wide): a box the exact test
// accepts is accepted here too, so no primitive is missed; only the visiting order differs from
// the binary SAH walk (closest hit: equal-distance ties; any hit: no change).  Stack entries are
// child groups {first child << 8 | mask of pending children}: one entry per level.
__device__ __forceinline__ bool wbox(float lx, float ly, float lz, float hx, float hy, float hz, const Ray& r, const f3& inv,
                                     float tmin, float tmax, float& t0_out)
{
    return slab_box(lx, ly, lz, hx, hy, hz, r, inv, tmin, tmax, t0_out);
}
__device__ __forceinline__ float ubyte(uint32_t w, int k) { return (float)((w >> (8 * (k & 3))) & 0xffu); }

struct WideHits {
    uint32_t inner, leaf; // slot masks
    int      nearest;     // inner slot with the smallest entry distance
    float    t_rest;      // smallest entry distance of the other hit inner slots
    uint32_t child_base, leaf_base, meta_lo, meta_hi;
};
__device__ __forceinline__ WideHits wide_visit(const Scene& sc, uint32_t node, const Ray& ray, const f3& inv, float tmin,
                                               float tmax, uint32_t filter = 0xffu)
{
    const uint4*   np = sc.wnodes + 5 * (size_t)node;
    SP_TD(td_lines(TD_NODE, np, 80));
#if SP_XP_DUP >= 1
    uint4 w0 = np[0], w1 = np[1], w2 = np[2], w3 = np[3], w4 = np[4];
    xp_dup(np, w0, w1, w2, w3, w4);
#else
    const uint4    w0 = np[0], w1 = np[1], w2 = np[2], w3 = np[3], w4 = np[4];
#endif
    const float    px = __uint_as_float(w0.x), py = __uint_as_float(w0.y), pz = __uint_as_float(w0.z);
    const float    sx = __uint_as_float((w0.w & 0xffu) << 23);
    const float    sy = __uint_as_float(((w0.w >> 8) & 0xffu) << 23);
    const float    sz = __uint_as_float(((w0.w >> 16) & 0xffu) << 23);
    const uint32_t imask = w0.w >> 24;
    WideHits       r;
    r.inner = 0; r.leaf = 0; r.nearest = -1; r.t_rest = k_infinite;
    r.child_base = w1.x; r.leaf_base = w1.y; r.meta_lo = w1.z; r.meta_hi = w1.w;
    float best = k_infinite;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        const uint32_t meta  = ((k < 4 ? w1.z : w1.w) >> (8 * (k & 3))) & 0xffu;
        const bool     inner = (imask >> k) & 1u;
        if (!inner && meta == 0u) continue;
        if (!((filter >> k) & 1u)) continue;
        const int   h  = k >> 2;
        const float lx = fma_f(ubyte(h ? w2.y : w2.x, k), sx, px);
        const float ly = fma_f(ubyte(h ? w2.w : w2.z, k), sy, py);
        const float lz = fma_f(ubyte(h ? w3.y : w3.x, k), sz, pz);
        const float hx = fma_f(ubyte(h ? w3.w : w3.z, k), sx, px);
        const float hy = fma_f(ubyte(h ? w4.y : w4.x, k), sy, py);
        const float hz = fma_f(ubyte(h ? w4.w : w4.z, k), sz, pz);
        float       t0;
        if (!wbox(lx, ly, lz, hx, hy, hz, ray, inv, tmin, tmax, t0)) continue;
        if (inner) {
            r.inner |= 1u << k;
            if (t0 < best) { r.t_rest = best; best = t0; r.nearest = k; }
            else r.t_rest = std_min(r.t_rest, t0);
        } else {
            r.leaf |= 1u << k;
        }
    }
    return r;
}

__device__ __forceinline__ uint32_t key_mask(uint32_t m, uint32_t o);
// occ (walk cache, SP_OCC_CACHE): the wide slot of the primitive that occluded this lane's previous
// shadow ray.  It is tested first; if it occludes this ray too, the answer (an OR over every
// primitive the ray meets in [tmin, tmax]) is true without a walk.  A hit found by the walk
// becomes the new cached occluder.  Same answer either way: only which primitives are tested changes
// -- PROVIDED the walk would have reached the cached primitive, i.e. no box on the way to its leaf
// is rejected by wbox for a ray that tri_hit accepts in [tmin, tmax].  The quantised boxes are
// rounded outward (supersets), but the slab t and the Moller-Trumbore t round differently, so for a
// primitive lying in a box face, hit at t within an ulp or so of tmax, the walk can miss what the
// cache finds.  The cache relies on that edge case not arising; it is off by default since round 6
// (level on every DirectLighting config, profiles/r05/walk_cache/), so the default walk is exact.
__device__ __forceinline__ bool wide_any(const Scene& sc, const Ray& ray, float tmin, float tmax, Stack st,
                                         uint32_t* occ = nullptr)
{
    if (occ && *occ != 0xffffffffu && prim_any(sc, *occ, ray, tmin, tmax, sc.wslot_tri)) return true;
    const f3       inv = mk(1.0f / ray.d.x, 1.0f / ray.d.y, 1.0f / ray.d.z);
    const uint32_t o   = dir_sign_bits(ray.d);
    int            sp  = 0;
    uint32_t       node = 0;
    while (true) {
#ifdef SP_WAVE_PROF
        const uint64_t t_it = __builtin_amdgcn_s_memtime(); // region 7: any-hit walk steps
#define SP_WPROF_ANY wprof_end(7, t_it)
#else
#define SP_WPROF_ANY
#endif
        const WideHits wh = wide_visit(sc, node, ray, inv, tmin, tmax);
        for (uint32_t m = wh.leaf; m; m &= m - 1) {
            const int      k    = __ffs(m) - 1;
            const uint32_t meta = ((k < 4 ? wh.meta_lo : wh.meta_hi) >> (8 * (k & 3))) & 0xffu;
            const uint32_t base = wh.leaf_base + (meta & 31u);
            for (uint32_t j = 0; j < (meta >> 5); ++j)
                if (prim_any(sc, base + j, ray, tmin, tmax, sc.wslot_tri)) {
                    SP_WPROF_ANY;
                    if (occ) *occ = base + j;
                    return true;
                }
        }
        SP_WPROF_ANY;
        if (wh.inner) {
            const uint32_t rest = key_mask(wh.inner & ~(1u << wh.nearest), o); // octant order
            if (rest) {
                st.s[sp * 64 + st.lane] = (wh.child_base << 8) | rest;
                ++sp;
            }
            node = wh.child_base + (uint32_t)wh.nearest;
            continue;
        }
        if (sp == 0) break;
        const uint32_t e = st.s[(sp - 1) * 64 + st.lane];
        uint32_t       m = e & 0xffu;
        const int      k = __ffs(m) - 1;
        m &= m - 1;
        if (m) st.s[(sp - 1) * 64 + st.lane] = (e & ~0xffu) | m;
        else --sp;
        node = (e >> 8) + ((uint32_t)k ^ o);
    }
    return false;
}

// An 8-bit slot mask in visiting order for a ray with direction sign bits o: bit k of the result
// is slot k ^ o (sp_bvh.cpp places children by octant, so key order is roughly near to far).
__device__ __forceinline__ uint32_t key_mask(uint32_t m, uint32_t o)
{
    m = (o & 1u) ? (((m & 0x55u) << 1) | ((m >> 1) & 0x55u)) : m;
    m = (o & 2u) ? (((m & 0x33u) << 2) | ((m >> 2) & 0x33u)) : m;
    m = (o & 4u) ? (((m & 0x0fu) << 4) | ((m >> 4) & 0x0fu)) : m;
    return m;
}

// Closest hit over the 8-wide BVH: at each node the hit leaves' primitives are tested, the
// nearest hit inner child is entered and the other hit inner children are pushed as one group
// entry {child_base << 8 | key mask} with the group's smallest entry distance in the stack's
// upper half (s[(e + depth / 2) * 64 + lane]; the upload sizes the stack for it); a group whose distance exceeds the closest hit found since is
// dropped whole.  Every primitive whose (outward-rounded) box meets [tmin, t_closest] is tested,
// so the result is the binary walk's except which of two primitives at exactly equal t wins
// (here: the lower wide slot, prim_closest_w).
__device__ __forceinline__ Hit wide_closest(const Scene& sc, const Ray& ray, float tmin, Hit h, Stack st)
{
    const f3       inv = mk(1.0f / ray.d.x, 1.0f / ray.d.y, 1.0f / ray.d.z);
    const uint32_t o   = dir_sign_bits(ray.d);
    const int      half = st.depth >> 1;
    int            sp   = 0;
    uint32_t       node = 0;
    while (true) {
#ifdef SP_WAVE_PROF
        const uint64_t t_it = __builtin_amdgcn_s_memtime(); // region 6: closest-hit walk steps
#endif
        const WideHits wh = wide_visit(sc, node, ray, inv, tmin, h.t);
        for (uint32_t m = wh.leaf; m; m &= m - 1) {
            const int      k    = __ffs(m) - 1;
            const uint32_t meta = ((k < 4 ? wh.meta_lo : wh.meta_hi) >> (8 * (k & 3))) & 0xffu;
            const uint32_t base = wh.leaf_base + (meta & 31u);
            for (uint32_t j = 0; j < (meta >> 5); ++j) prim_closest_w(sc, base + j, ray, tmin, h);
        }
#ifdef SP_WAVE_PROF
        wprof_end(6, t_it);
#endif
        if (wh.inner) {
            const uint32_t rest = key_mask(wh.inner & ~(1u << wh.nearest), o);
            if (rest) {
                st.s[sp * 64 + st.lane]              = (wh.child_base << 8) | rest;
                st.s[(sp + half) * 64 + st.lane]    = __float_as_uint(wh.t_rest);
                ++sp;
            }
            node = wh.child_base + (uint32_t)wh.nearest;
            continue;
        }
        bool found = false;
        while (sp > 0) {
            const uint32_t e = st.s[(sp - 1) * 64 + st.lane];
            if (__uint_as_float(st.s[(sp - 1 + half) * 64 + st.lane]) > h.t) { --sp; continue; }
            uint32_t  m = e & 0xffu;
            const int k = __ffs(m) - 1;
            m &= m - 1;
            if (m) st.s[(sp - 1) * 64 + st.lane] = (e & ~0xffu) | m;
            else --sp;
            node  = (e >> 8) + ((uint32_t)k ^ o);
            found = true;
            break;
        }
        if (!found) break;
    }
    return h;
}

// ---------------------------------------------------------------- merged query pass
// Once a bounce's served estimates are taken, a live lane holds two ray queries that depend on
// nothing else still to come: the MIS ray of its (last) light's estimate_direct_mis
// (Integrator.cpp:527-533: intersect_lights, then intersect_p) and the next bounce's closest hit
// (:558-563, direction fixed at :570).  In lock step each was a wave-wide walk as long as its
// slowest lane's, at the occupancy of the paths still alive (0.59-0.67).  Here the cheap parts
// stay with the owner (the light tests, the unbounded shapes) and the BVH walks are posted to LDS
// and shared by every lane of the wave, ended paths included:
//   * each lane takes a query from the wave's queue and walks it (8-wide nodes, the octant order
//     and group stack of wide_closest / wide_any);
//   * a lane with nothing left to walk takes pending work from one that has: the OLDEST group entry
//     of its stack (the bottom -- the biggest subtree still unvisited), and walks it for that
//     query.  Pairs are dealt by lane order once per step, one thief per victim, so no two lanes
//     ever touch one stack entry; the lanes' steps are one SIMT instruction stream, and each
//     lane's stack bounds [bot, top) live in LDS (MQ_TB) for its thief.
// A closest-hit query's answer is the lexicographic minimum of (t, wide slot) over every primitive
// it hits (prim_closest_w: independent of which lane meets which primitive first); the lanes
// sharing it meet in one u64 atomicMin (MQ_BEST), which also gives every one of them the current
// t_max for its box tests and group culling.  An any-hit query ends for everyone once one lane
// finds a hit (MQ_ANY); its t_max is FLT_MAX, so nothing is culled for it, as in wide_any.
// Results are the per-lane walks' (SP_RENDER_PER_LANE_QUERIES: bit-identical images and counts);
// only which lane walks which node changes.
__device__ __forceinline__ float    mq_f(const uint32_t* m, int i) { return __uint_as_float(m[i]); }
__device__ __forceinline__ f3       mq_f3(const uint32_t* m, int b, int o) { return mk(mq_f(m, b + o), mq_f(m, b + 64 + o), mq_f(m, b + 128 + o)); }
__device__ __forceinline__ void     mq_put3(uint32_t* m, int b, int o, f3 v)
{
    m[b + o]       = __float_as_uint(v.x);
    m[b + 64 + o]  = __float_as_uint(v.y);
    m[b + 128 + o] = __float_as_uint(v.z);
}
template <class L>
__device__ __forceinline__ unsigned long long* mq_best(uint32_t* m, int o)
{
    return reinterpret_cast<unsigned long long*>(m + L::BEST) + o;
}
__device__ __forceinline__ void mq_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
#ifndef SP_MQ_STEAL
#define SP_MQ_STEAL 1
#endif
// The per-wave LDS rows a shared walk uses: L::O / D3 / T3 the any-hit rays (origin, direction,
// t_min), L::AMAX their t_max, L::ANY their results; L::D1 / T1 the closest-hit rays (origin in
// L::O too), L::BEST their u64 (t, wide slot) answers; L::TB the walking lanes' stack bounds and
// queries, L::Q the queue (query r = owner lane | any-hit << 7), L::CNT its next unclaimed entry.
// All lanes in integrate() call it; total = queries in m[L::Q..] (posted and synchronised by the
// caller).  any_tmax: any-hit queries' t_max is in m[L::AMAX + owner]; else FLT_MAX (MIS rays).
// ANY_ONLY: no closest-hit query is ever posted (the closest-hit code is not compiled).
#ifndef SP_MQ_PAIRS // thief / victim pairs dealt per walk step: elf 1024^2 @ 16 spp 879-884 at 8, 890-893 at 16 and 64
#define SP_MQ_PAIRS 16
#endif
template <class L, bool ANY_ONLY = false>
__device__ __forceinline__ void mq_run(const Scene& sc, Stack st, uint32_t* m, int total, bool any_tmax = false)
{
    const int      lane = threadIdx.x & 63;
    const uint64_t lt   = (1ull << lane) - 1ull;
    const uint64_t act  = __ballot(1);
    int            q    = __popcll(act & lt); // first round: one query per lane present
    if (q == 0) m[L::CNT] = (uint32_t)__popcll(act);
    mq_sync();
    const int      half = st.depth >> 1;
    const uint8_t* qs   = reinterpret_cast<const uint8_t*>(m + L::Q);
    // the lane's walk: query (owner, any), node to visit, its stack [bot, sp)
    Ray      ray;
    f3       inv  = mk(0, 0, 0);
    uint32_t o    = 0, node = 0;
    float    tmin = 0.0f, amax = k_infinite;
    bool     any  = false, has_node = false;
    int      own  = -1, sp = 0, bot = 0;
    auto load = [&](uint32_t e) { // query e = owner | any << 6
        own   = (int)(e & 63u);
        any   = ANY_ONLY || (e & 64u) != 0u;
        ray.o = mq_f3(m, L::O, own);
        ray.d = mq_f3(m, any ? L::D3 : L::D1, own);
        tmin  = mq_f(m, (any ? L::T3 : L::T1) + own);
        amax  = (any && any_tmax) ? mq_f(m, L::AMAX + own) : k_infinite;
        inv   = mk(1.0f / ray.d.x, 1.0f / ray.d.y, 1.0f / ray.d.z);
        o     = dir_sign_bits(ray.d);
    };
    auto take = [&](int qi) {
        const uint32_t e = qs[qi];
        load((e & 63u) | ((e >> 1) & 64u));
        node = 0; has_node = true; sp = 0; bot = 0;
        m[L::TB + lane] = ((uint32_t)own << 16) | (any ? 1u << 22 : 0u);
    };
    if (q < total) take(q);
    while (true) {
        if (own >= 0) {
#ifdef SP_WAVE_PROF
            const uint64_t t_it = __builtin_amdgcn_s_memtime(); // region 4: lanes walking, per step
#endif
            bot = (int)((m[L::TB + lane] >> 8) & 0xffu); // a thief may have raised it
            float tmax;
            if (any) {
                tmax = amax;
                if (m[L::ANY + own] != 0u) { has_node = false; sp = bot; } // another lane found a hit
            } else {
                if constexpr (!ANY_ONLY) tmax = __uint_as_float((uint32_t)(*mq_best<L>(m, own) >> 32));
                else tmax = amax;
            }
            if (!has_node) { // the next pending group child, culled by the current closest t
                while (sp > bot) {
                    const uint32_t e = st.s[(sp - 1) * 64 + st.lane];
                    if (__uint_as_float(st.s[(sp - 1 + half) * 64 + st.lane]) > tmax) { --sp; continue; }
                    uint32_t  mk8 = e & 0xffu;
                    const int k   = __ffs(mk8) - 1;
                    mk8 &= mk8 - 1;
                    if (mk8) st.s[(sp - 1) * 64 + st.lane] = (e & ~0xffu) | mk8;
                    else --sp;
                    node     = (e >> 8) + ((uint32_t)k ^ o);
                    has_node = true;
                    break;
                }
            }
            if (has_node) {
                const WideHits wh    = wide_visit(sc, node, ray, inv, tmin, tmax);
                bool           found = false;
                Hit            h;
                h.t = tmax; h.code = 0xffffffffu; h.beta = h.gamma = 0.0f; h.slot = 0xffffffffu;
                for (uint32_t mm = wh.leaf; mm && !found; mm &= mm - 1) {
                    const int      k    = __ffs(mm) - 1;
                    const uint32_t meta = ((k < 4 ? wh.meta_lo : wh.meta_hi) >> (8 * (k & 3))) & 0xffu;
                    const uint32_t base = wh.leaf_base + (meta & 31u);
                    for (uint32_t j = 0; j < (meta >> 5); ++j) {
                        if (any) {
                            if (prim_any(sc, base + j, ray, tmin, tmax, sc.wslot_tri)) { found = true; break; }
                        } else if constexpr (!ANY_ONLY) {
                            prim_closest_w(sc, base + j, ray, tmin, h); // the lane's minimum over the node
                        }
                    }
                }
                if constexpr (!ANY_ONLY) {
                    if (!any && h.slot != 0xffffffffu)
                        atomicMin(mq_best<L>(m, own), ((unsigned long long)__float_as_uint(h.t) << 32) | h.slot);
                }
                if (found) {
                    m[L::ANY + own] = 1u;
                    has_node = false;
                    sp       = bot;
                } else if (wh.inner) {
                    const uint32_t rest = key_mask(wh.inner & ~(1u << wh.nearest), o); // octant order
                    if (rest) {
                        st.s[sp * 64 + st.lane]          = (wh.child_base << 8) | rest;
                        st.s[(sp + half) * 64 + st.lane] = __float_as_uint(wh.t_rest);
                        ++sp;
                    }
                    node = wh.child_base + (uint32_t)wh.nearest;
                } else {
                    has_node = false;
                }
            }
            if (!has_node && sp == bot) own = -1; // this lane's part of the query is done
            m[L::TB + lane] = (uint32_t)sp | ((uint32_t)bot << 8) | ((uint32_t)(own & 63) << 16) | (any ? 1u << 22 : 0u);
#ifdef SP_WAVE_PROF
            wprof_end(4, t_it);
#endif
        }
        if (own < 0 && (int)m[L::CNT] < total) { // the queue first
            const int qi = (int)atomicAdd(&m[L::CNT], 1u);
            if (qi < total) take(qi);
        }
        const uint64_t idle = __ballot(own < 0);
        if (idle == act) break; // nothing walked, nothing pending, queue empty
#if SP_MQ_STEAL
        uint64_t can = __ballot(own >= 0 && sp > bot); // lanes with a pending group entry
        if (idle != 0ull && can != 0ull) {
            mq_sync(); // the victims' stacks and bounds are in LDS
            // pair idle lanes with victims in lane order (one thief per victim)
            uint64_t ii = idle;
            int      vict = -1;
            for (int k = 0; k < SP_MQ_PAIRS && ii != 0ull && can != 0ull; ++k) {
                const int v = __ffsll((unsigned long long)can) - 1, t = __ffsll((unsigned long long)ii) - 1;
                can &= can - 1ull;
                ii &= ii - 1ull;
                if (lane == t) vict = v;
            }
            if (vict >= 0) {
                const uint32_t tb = m[L::TB + vict];
                const int      vb = (int)((tb >> 8) & 0xffu);
                const uint32_t e  = st.s[vb * 64 + vict];
                const uint32_t dd = st.s[(vb + half) * 64 + vict];
                m[L::TB + vict]   = (tb & ~0xff00u) | ((uint32_t)(vb + 1) << 8);
                load(((tb >> 16) & 63u) | ((tb >> 16) & 64u));
                st.s[st.lane]          = e; // the stolen group is this lane's whole stack
                st.s[half * 64 + st.lane] = dd;
                sp = 1; bot = 0; has_node = false;
                m[L::TB + lane] = 1u | ((uint32_t)own << 16) | (any ? 1u << 22 : 0u);
            }
            mq_sync();
        }
#endif
    }
    mq_sync();
}

// Wave-uniform record fetch through the constant address space: with the address in SGPRs
// the compiler emits s_load (scalar cache).  A uniform-address VECTOR load still costs the
// vector L1 a per-lane access (TCP_TOTAL_ACCESSES), which is what bounds the traversal kernels.
// Only for records whose index is equal across the active lanes (loops over scene lists).
typedef const __attribute__((address_space(4))) float    cf32;
typedef const __attribute__((address_space(4))) uint32_t cu32;
__device__ __forceinline__ uintptr_t uptr(const void* p)
{
    const uint64_t a  = (uint64_t)(uintptr_t)p;
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)a);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(a >> 32));
    return (uintptr_t)(((uint64_t)hi << 32) | lo);
}
__device__ __forceinline__ uint32_t uload_u32(const void* p) { return *(cu32*)uptr(p); }
__device__ __forceinline__ f3 uload_f3(const f3* p)
{
    cf32* q = (cf32*)uptr(p);
    return mk(q[0], q[1], q[2]);
}
__device__ __forceinline__ aff uload_aff(const aff* p)
{
    aff a;
    a.vx = uload_f3(&p->vx);
    a.vy = uload_f3(&p->vy);
    a.vz = uload_f3(&p->vz);
    a.p  = uload_f3(&p->p);
    return a;
}
__device__ __forceinline__ Node uload_node(const Node* p)
{
    cu32* q = (cu32*)uptr(p);
    Node  n;
    n.lo[0] = __uint_as_float(q[0]); n.lo[1] = __uint_as_float(q[1]); n.lo[2] = __uint_as_float(q[2]); n.a = q[3];
    n.hi[0] = __uint_as_float(q[4]); n.hi[1] = __uint_as_float(q[5]); n.hi[2] = __uint_as_float(q[6]); n.b = q[7];
    return n;
}
// the fields of a sphere / sphere light that ray tests read
struct UShape {
    aff     w2o;
    int32_t kind;
};
__device__ __forceinline__ UShape uload_shape(const Shape* p)
{
    UShape u;
    u.w2o  = uload_aff(&p->w2o);
    u.kind = (int32_t)uload_u32(&p->kind);
    return u;
}
__device__ __forceinline__ Light uload_light(const Light* p)
{
    Light l;
    l.kind     = (int32_t)uload_u32(&p->kind);
    l.image    = (int32_t)uload_u32(reinterpret_cast<const uint32_t*>(&p->image));
    const f3 r = uload_f3(reinterpret_cast<const f3*>(&p->radiance));
    l.radiance = mkc(r.x, r.y, r.z);
    l.o2w      = uload_aff(&p->o2w);
    l.w2o      = uload_aff(&p->w2o);
    l.nrm.vx   = uload_f3(&p->nrm.vx);
    l.nrm.vy   = uload_f3(&p->nrm.vy);
    l.nrm.vz   = uload_f3(&p->nrm.vz);
    return l;
}

// BVHAccelerator::intersect (shapes/BVHAccelerator.h:62-77) over the binary BVH
template <bool SL>
__device__ __forceinline__ Hit bvh_closest(const Scene& sc, const Ray& ray, float tmin, Hit h, Stack st)
{
    const f3 inv = mk(1.0f / ray.d.x, 1.0f / ray.d.y, 1.0f / ray.d.z);
    BinWalk<SL> w = bin_walk<SL>(st, sc.nodes, sc.parents, sc.ordered != 0, ray.d);
    uint32_t cur = 0;      // root: no box test
    bool     test_box = false;
    while (true) {
        const Node n = sc.nodes[cur];
        if (!test_box || box_hit(n, ray, inv, tmin, h.t)) {
            if (n.b & LEAF_BIT) {
                const uint32_t cnt = n.b & ~LEAF_BIT;
                for (uint32_t k = 0; k < cnt; ++k) prim_closest(sc, n.a + k, ray, tmin, h);
            } else {
                uint32_t first, second; // reference: child 0 first
                children_in_order(w, n, ray.d, first, second);
                walk_defer(w, second); // box tested when the walk comes back to it
                cur      = first;
                test_box = true;
                continue;
            }
        }
        if (!walk_next(w, ray.d, cur)) break;
        test_box = true;
    }
    return h;
}

// Scene::intersect (base/Scene.h:74): ListAccelerator{unbounded..., BVH} -- the unbounded shapes
__device__ __forceinline__ Hit scene_intersect_unbounded(const Scene& sc, const Ray& ray, float tmin, float tmax)
{
    Hit h;
    h.t    = tmax;
    h.code = 0xffffffffu;
    for (int i = 0; i < sc.n_unbounded; ++i) {
        const int    sid = (int)uload_u32(sc.unbounded + i);
        const UShape s   = uload_shape(sc.shapes + sid);
        float        t;
        const bool  hit = (s.kind == SP_PRIM_SPHERE) ? sphere_t(s.w2o, ray, tmin, h.t, t) : plane_t(s.w2o, ray, tmin, h.t, t);
        if (hit) { h.t = t; h.code = ((uint32_t)s.kind << CODE_SHIFT) | (uint32_t)sid; }
    }
    return h;
}
__device__ __forceinline__ Hit scene_intersect(const Scene& sc, const Ray& ray, float tmin, float tmax, Stack st)
{
    Hit h = scene_intersect_unbounded(sc, ray, tmin, tmax);
    if (sc.n_nodes == 0) return h;
    if (sc.wide_closest) return wide_closest(sc, ray, tmin, h, st);
    return sc.stackless ? bvh_closest<true>(sc, ray, tmin, h, st) : bvh_closest<false>(sc, ray, tmin, h, st);
}

// BVHAccelerator::intersect_p over the binary BVH
template <bool SL>
__device__ __forceinline__ bool bvh_any(const Scene& sc, const Ray& ray, float tmin, float tmax, Stack st)
{
    const f3 inv = mk(1.0f / ray.d.x, 1.0f / ray.d.y, 1.0f / ray.d.z);
    BinWalk<SL> w = bin_walk<SL>(st, sc.nodes, sc.parents, sc.ordered != 0, ray.d);
    uint32_t cur = 0;
    bool     test_box = false;
    while (true) {
        const Node n = sc.nodes[cur];
        if (!test_box || box_hit(n, ray, inv, tmin, tmax)) {
            if (n.b & LEAF_BIT) {
                const uint32_t cnt = n.b & ~LEAF_BIT;
                for (uint32_t k = 0; k < cnt; ++k)
                    if (prim_any(sc, n.a + k, ray, tmin, tmax)) return true;
            } else {
                uint32_t first, second;
                children_in_order(w, n, ray.d, first, second);
                walk_defer(w, second);
                cur      = first;
                test_box = true;
                continue;
            }
        }
        if (!walk_next(w, ray.d, cur)) break;
        test_box = true;
    }
    return false;
}

// any-hit over the geometry accelerator (ListAccelerator::intersect_p_impl): the unbounded shapes
__device__ __forceinline__ bool unbounded_any(const Scene& sc, const Ray& ray, float tmin, float tmax)
{
    for (int i = 0; i < sc.n_unbounded; ++i) {
        const UShape s = uload_shape(sc.shapes + uload_u32(sc.unbounded + i));
        float        t;
        if ((s.kind == SP_PRIM_SPHERE) ? sphere_t(s.w2o, ray, tmin, tmax, t) : plane_t(s.w2o, ray, tmin, tmax, t)) return true;
    }
    return false;
}
__device__ __forceinline__ bool geometry_any(const Scene& sc, const Ray& ray, float tmin, float tmax, Stack st,
                                             uint32_t* occ = nullptr)
{
    if (unbounded_any(sc, ray, tmin, tmax)) return true;
    if (sc.n_nodes == 0) return false;
    if (sc.wnodes) return wide_any(sc, ray, tmin, tmax, st, occ);
    return sc.stackless ? bvh_any<true>(sc, ray, tmin, tmax, st) : bvh_any<false>(sc, ray, tmin, tmax, st);
}

// ------------------------------------------------------------------------------ image environment light
// ImageBasedEnvironmentLight (Lights/Light.h:196) on the device.  The tables are the ones its
// constructor builds (sp_envmap.cpp); the lookups below restate Distribution1D/2D sampling and
// the nearest-neighbour texel fetch with the reference's operation order.

// Distribution1D::get_offset (math/Distribution1D.h:130): libstdc++ ranges::upper_bound over the
// n + 1 cdf entries, step for step (the last entry is the integral, not 1, so the array is not
// sorted and only this exact search reproduces the reference's offsets).
__device__ __forceinline__ int dist_offset(const float* cdf, int n, float u)
{
    int first = 0, len = n + 1;
    while (len > 0) {
        const int half = len >> 1;
        const int mid  = first + half;
        if (u < cdf[mid]) {
            len = half;
        } else {
            first = mid + 1;
            len   = len - half - 1;
        }
    }
    return (first >= n) ? n - 1 : first; // it == end() || it == prev(end())
}
// The same offset through a guide table (sp_host.hpp EnvMap): cdf[0..n-1] is non-decreasing, so
// the replayed search returns the first i < n with u < cdf[i] (else n - 1); the guide narrows it
// to [guide[b], guide[b+1]] for b = floor(u * 2^bits) (exact: power-of-two scale), usually one
// or two entries, instead of 13 dependent probes over a 32 KB row.
__device__ __forceinline__ int dist_offset_guided(const float* cdf, const uint32_t* guide, int bits, float u)
{
    const int b  = (int)(u * (float)(1 << bits));
    int       lo = (int)guide[b], hi = (int)guide[b + 1];
    while (lo < hi) {
        const int mid = (lo + hi) >> 1;
        if (u < cdf[mid]) hi = mid;
        else lo = mid + 1;
    }
    return lo;
}
// Distribution1D::sample_continuous (math/Distribution1D.h:72) on [0, 1]
__device__ __forceinline__ float dist_sample(const float* func, const float* cdf, int n, float integral, float u, float& pdf,
                                             int& off, const uint32_t* guide = nullptr, int bits = 0)
{
    off            = guide ? dist_offset_guided(cdf, guide, bits, u) : dist_offset(cdf, n, u);
    const float c0 = cdf[off], c1 = cdf[off + 1];
    float       du = u - c0;
    if ((c1 - c0) > 0.0f) du /= (c1 - c0);
    pdf           = (integral > 0.0f) ? func[off] / integral : 0.0f;
    const float x = (static_cast<float>(off) + du) / static_cast<float>(n);
    return (1.0f - x) * 0.0f + x * 1.0f; // lerp(x, m_min, m_max)
}
// static_cast<std::size_t>(x) clamped to [0, n - 1] as x86-64 GCC converts (negative <= -1 and
// NaN wrap to huge values, which the clamp maps to n - 1).
__device__ __forceinline__ int size_clamp(float x, int n)
{
    if (x >= 0.0f) return (x >= static_cast<float>(n)) ? n - 1 : static_cast<int>(x);
    return (x > -1.0f) ? 0 : n - 1;
}
// sample_nearest_neighbor(img, s, t, RemapWrap, RemapClamp) (Image/Image.h:99)
__device__ __forceinline__ rgb env_texel(const EnvMap& e, float s, float t)
{
    s                = fmod1(1.0f + fmod1(s));
    t                = std_clamp(t, 0.0f, 0x1.fffffep-1f);
    const float    u = round_f(s * static_cast<float>(e.w));
    const float    v = round_f(t * static_cast<float>(e.h));
    const uint32_t x = min(static_cast<uint32_t>(u), static_cast<uint32_t>(e.w - 1));
    const uint32_t y = min(static_cast<uint32_t>(v), static_cast<uint32_t>(e.h - 1));
    const float4   c = e.radiance[(size_t)y * (uint32_t)e.w + x];
    return mkc(c.x, c.y, c.z);
}
// spherical_theta / spherical_phi (math/Sampling.h:82-91)
__device__ __forceinline__ float spherical_theta(f3 v) { return lm_acosf(std_clamp(v.y, -1.0f, 1.0f)); }
__device__ __forceinline__ float spherical_phi(f3 v)
{
    const float p = lm_atan2f(v.z, v.x);
    return (p < 0.0f) ? (p + 2.0f * k_pi) : p;
}
constexpr float k_inv_2_pi = 1.0f / (2.0f * k_pi);
// ImageBasedEnvironmentLight::intersect_lights_impl radiance (Lights/Light.h:216)
__device__ __forceinline__ rgb env_radiance(const EnvMap& e, f3 dir, const Rsq& q)
{
    const f3 w = normalize(xfm_vector(e.w2l, dir), q);
    return env_texel(e, spherical_phi(w) * k_inv_2_pi, spherical_theta(w) * k_inv_pi);
}
struct EnvSample {
    rgb   L;
    float pdf;
    f3    wi;
};
// ImageBasedEnvironmentLight::light_sample (Lights/Light.h:243)
__device__ __forceinline__ EnvSample env_sample(const EnvMap& e, P2 u)
{
    EnvSample s;
    float     pdf1, pdf0;
    int       v, iu;
    const float d1 = dist_sample(e.marg_func, e.marg_cdf, e.nv, e.marg_int, u.y, pdf1, v, e.marg_guide, e.marg_bits);
    const uint32_t* cg = e.cond_guide ? e.cond_guide + (size_t)v * ((1u << e.cond_bits) + 1u) : nullptr;
    const float d0 = dist_sample(e.cond_func + (size_t)v * e.nu, e.cond_cdf + (size_t)v * (e.nu + 1), e.nu, e.cond_int[v], u.x,
                                 pdf0, iu, cg, e.cond_bits);
    const float map_pdf = pdf0 * pdf1;
    if (map_pdf == 0.0f) {
        s.L   = mkc(0, 0, 0);
        s.pdf = 0.0f;
        s.wi  = mk(0, 0, 0);
        return s;
    }
    const float theta     = d1 * k_pi;
    const float phi       = d0 * 2.0f * k_pi;
    float       sin_theta, cos_theta, sin_phi, cos_phi;
    lm_sincosf(theta, &sin_theta, &cos_theta);
    lm_sincosf(phi, &sin_phi, &cos_phi);
    s.wi  = xfm_vector(e.l2w, mk(sin_theta * cos_phi, cos_theta, sin_theta * sin_phi));
    s.pdf = (sin_theta == 0.0f) ? 0.0f : map_pdf / (2.0f * (k_pi * k_pi) * sin_theta);
    s.L   = env_texel(e, d0, d1);
    return s;
}
// ImageBasedEnvironmentLight::pdf_impl (Lights/Light.h:270); note the reference passes
// theta * pi (not theta / pi) as the second coordinate to Distribution2D::pdf.
__device__ __forceinline__ float env_pdf(const EnvMap& e, f3 wi)
{
    const f3    w         = xfm_vector(e.w2l, wi);
    const float theta     = spherical_theta(w);
    const float phi       = spherical_phi(w);
    const float sin_theta = lm_sinf(theta);
    if (sin_theta == 0.0f) return 0.0f;
    const int iu = size_clamp(phi * k_inv_2_pi * static_cast<float>(e.nu), e.nu);
    const int iv = size_clamp(theta * k_pi * static_cast<float>(e.nv), e.nv);
    return (e.cond_func[(size_t)iv * e.nu + iu] / e.marg_int) / (2.0f * (k_pi * k_pi) * sin_theta);
}

// ------------------------------------------------------------------------------ lights
struct LightHit {
    bool    hit;
    float   t;
    rgb     L;   // radiance of the light hit (constant lights)
    int32_t env; // >= 0: an image environment light won; its radiance depends on the direction
};
// LightIntersection::L of a hit (light_hit_L evaluates an image light lazily: the integrators
// only read L when no geometry is in front of the light).

// the sphere lights' BVH (child 0 first: reference build)
template <bool SL>
__device__ __forceinline__ LightHit light_bvh_closest(const Scene& sc, const Ray& ray, float tmin, LightHit lh, Stack st)
{
    const f3 inv = mk(1.0f / ray.d.x, 1.0f / ray.d.y, 1.0f / ray.d.z);
    BinWalk<SL> w = bin_walk<SL>(st, sc.light_nodes, sc.light_parents, false, ray.d);
    uint32_t cur = 0;
    bool     test_box = false;
    while (true) {
        const Node n = sc.light_nodes[cur];
        if (!test_box || box_hit(n, ray, inv, tmin, lh.t)) {
            if (n.b & LEAF_BIT) {
                const uint32_t cnt = n.b & ~LEAF_BIT;
                for (uint32_t k = 0; k < cnt; ++k) {
                    const Light& l = sc.lights[sc.light_slot[n.a + k]];
                    float        t;
                    if (sphere_t(l.w2o, ray, tmin, lh.t, t)) {
                        lh.hit = true;
                        lh.t   = t;
                        lh.L   = l.radiance;
                        lh.env = -1;
                    }
                }
            } else {
                walk_defer(w, n.b);
                cur      = n.a & CHILD_MASK;
                test_box = true;
                continue;
            }
        }
        if (!walk_next(w, ray.d, cur)) break;
        test_box = true;
    }
    return lh;
}

// Scene::intersect_lights (base/Scene.h:69): ListAccelerator{environment..., BVH(sphere lights)}
__device__ __forceinline__ LightHit scene_intersect_lights(const Scene& sc, const Ray& ray, float tmin, float tmax, Stack st)
{
    LightHit lh;
    lh.hit = false;
    lh.t   = tmax;
    lh.env = -1;
    for (int i = 0; i < sc.n_unbounded_lights; ++i) {
        const Light l = uload_light(sc.lights + uload_u32(sc.unbounded_lights + i));
        // EnvironmentLight / ImageBasedEnvironmentLight::intersect_lights_impl (Lights/Light.h:152, :206)
        if (!(lh.t < k_infinite)) {
            lh.hit = true;
            lh.t   = k_infinite;
            lh.L   = l.radiance;
            lh.env = (l.kind == SP_LIGHT_IMAGE_ENVIRONMENT) ? l.image : -1;
        }
    }
    if (sc.n_light_nodes == 0) return lh;
    if (sc.n_light_nodes == 1) { // a single leaf (root: no box test): the same lights for every lane
        const Node     n   = uload_node(sc.light_nodes);
        const uint32_t cnt = n.b & ~LEAF_BIT;
        for (uint32_t k = 0; k < cnt; ++k) {
            const Light* lp = sc.lights + uload_u32(sc.light_slot + n.a + k);
            const aff    w2o = uload_aff(&lp->w2o);
            float        t;
            if (sphere_t(w2o, ray, tmin, lh.t, t)) {
                const f3 r = uload_f3(reinterpret_cast<const f3*>(&lp->radiance));
                lh.hit = true;
                lh.t   = t;
                lh.L   = mkc(r.x, r.y, r.z);
                lh.env = -1;
            }
        }
        return lh;
    }
    return sc.stackless ? light_bvh_closest<true>(sc, ray, tmin, lh, st) : light_bvh_closest<false>(sc, ray, tmin, lh, st);
}

__device__ __forceinline__ rgb light_hit_L(const Scene& sc, const LightHit& lh, f3 dir, const Rsq& q)
{
    return (lh.env >= 0) ? env_radiance(sc.envs[lh.env], dir, q) : lh.L;
}

template <bool SL>
__device__ __forceinline__ bool light_bvh_any(const Scene& sc, const Ray& ray, float tmin, float tmax, Stack st)
{
    const f3 inv = mk(1.0f / ray.d.x, 1.0f / ray.d.y, 1.0f / ray.d.z);
    BinWalk<SL> w = bin_walk<SL>(st, sc.light_nodes, sc.light_parents, false, ray.d);
    uint32_t cur = 0;
    bool     test_box = false;
    while (true) {
        const Node n = sc.light_nodes[cur];
        if (!test_box || box_hit(n, ray, inv, tmin, tmax)) {
            if (n.b & LEAF_BIT) {
                const uint32_t cnt = n.b & ~LEAF_BIT;
                for (uint32_t k = 0; k < cnt; ++k) {
                    const Light& l = sc.lights[sc.light_slot[n.a + k]];
                    float        t;
                    if (sphere_t(l.w2o, ray, tmin, tmax, t)) return true;
                }
            } else {
                walk_defer(w, n.b);
                cur      = n.a & CHILD_MASK;
                test_box = true;
                continue;
            }
        }
        if (!walk_next(w, ray.d, cur)) break;
        test_box = true;
    }
    return false;
}

__device__ __forceinline__ bool lights_any(const Scene& sc, const Ray& ray, float tmin, float tmax, Stack st)
{
    if (sc.n_light_nodes == 0) return false; // environment lights never occlude
    if (sc.n_light_nodes == 1) {
        const Node     n   = uload_node(sc.light_nodes);
        const uint32_t cnt = n.b & ~LEAF_BIT;
        for (uint32_t k = 0; k < cnt; ++k) {
            const aff w2o = uload_aff(&sc.lights[uload_u32(sc.light_slot + n.a + k)].w2o);
            float     t;
            if (sphere_t(w2o, ray, tmin, tmax, t)) return true;
        }
        return false;
    }
    return sc.stackless ? light_bvh_any<true>(sc, ray, tmin, tmax, st) : light_bvh_any<false>(sc, ray, tmin, tmax, st);
}

// Scene::intersect_p (base/Scene.h:79)
__device__ __forceinline__ bool scene_any(const Scene& sc, const Ray& ray, float tmin, float tmax, Stack st,
                                          uint32_t* occ = nullptr)
{
    return geometry_any(sc, ray, tmin, tmax, st, occ) || lights_any(sc, ray, tmin, tmax, st);
}

// ------------------------------------------------------------------------------ sampling
// math/Sampling.h:222
__device__ __forceinline__ f3 sample_uniform_sphere(P2 u)
{
    const float z   = 1.0f - 2.0f * u.x;
    const float r   = sqrt_unit(std_max(0.0f, 1.0f - z * z));
    const float phi = (float)(2.0 * (double)k_pi * (double)u.y);
    float       sp, cp;
    lm_sincosf_bounded(phi, &sp, &cp); // u in [0, 1): |phi| < 2 pi
    return mk(r * cp, r * sp, z);
}
// math/Sampling.h:235
__device__ __forceinline__ f3 sample_uniform_hemisphere(P2 u)
{
    const float y   = u.x;
    const float r   = sqrt_unit(std_max(0.0f, 1.0f - y * y));
    const float phi = 2.0f * k_pi * u.y;
    float       sp, cp;
    lm_sincosf_bounded(phi, &sp, &cp); // u in [0, 1): |phi| < 2 pi
    return mk(r * cp, y, r * sp);
}
// math/Sampling.cpp:304
__device__ __forceinline__ P2 concentric_disk(P2 u)
{
    constexpr float pi_over_4 = k_pi / 4.0f;
    constexpr float pi_over_2 = k_pi / 2.0f;
    const float     ox = 2.0f * u.x - 1.0f;
    const float     oy = 2.0f * u.y - 1.0f;
    P2              r;
    if (ox == 0.0f && oy == 0.0f) { r.x = 0.0f; r.y = 0.0f; return r; }
    float theta, rad;
    if (abs_f(ox) > abs_f(oy)) { rad = ox; theta = pi_over_4 * (oy / ox); }
    else { rad = oy; theta = pi_over_2 - pi_over_4 * (ox / oy); }
    float st, ct;
    lm_sincosf_bounded(theta, &st, &ct); // |theta| <= 3 pi / 4
    r.x = rad * ct;
    r.y = rad * st;
    return r;
}
__device__ __forceinline__ f3 sample_cosine_hemisphere(P2 u)
{
    const P2    d = concentric_disk(u);
    const float y = sqrt_unit(std_max(0.0f, 1.0f - d.x * d.x - d.y * d.y)); // 0 or >= 2^-48
    return mk(d.x, y, d.y);
}
constexpr float k_uniform_sphere_pdf     = 1.0f / (4.0f * k_pi);
constexpr float k_uniform_hemisphere_pdf = 1.0f / (2.0f * k_pi);

// math/ONB.h
struct Onb {
    f3 u, v, w;
};
__device__ __forceinline__ Onb onb_of_unit(f3 v)
{
    const float sign = copysign_f(1.0f, v.z);
    const float a    = -1.0f / (sign + v.z);
    const float b    = v.x * v.y * a;
    const f3    b1   = mk(1.0f + sign * v.x * v.x * a, sign * b, -sign * v.x);
    const f3    b2   = mk(b, sign + v.y * v.y * a, -v.y);
    Onb         o;
    o.u = b2; // [w, u] = create(v)
    o.v = v;
    o.w = b1;
    return o;
}
__device__ __forceinline__ Onb onb_from_v(f3 n, const Rsq& q) { return onb_of_unit(normalize(n, q)); }
__device__ __forceinline__ f3 to_world(const Onb& o, f3 a) { return add(add(scale(a.x, o.u), scale(a.y, o.v)), scale(a.z, o.w)); }
__device__ __forceinline__ f3 to_onb(const Onb& o, f3 a) { return mk(dot(a, o.u), dot(a, o.v), dot(a, o.w)); }

// ------------------------------------------------------------------------------ materials
struct MSample {
    rgb   color;
    f3    dir;
    float pdf;
    int   props;
};
constexpr int PROP_DIFFUSE = 1, PROP_GLOSSY = 2, PROP_SPECULAR = 4, PROP_REFLECTIVE = 8;

__device__ __forceinline__ float cos2_theta(f3 w) { return w.y * w.y; }
__device__ __forceinline__ float sin2_theta(f3 w) { return std_max(0.0f, 1.0f - cos2_theta(w)); }
__device__ __forceinline__ float sin_theta(f3 w) { return sqrt_unit(sin2_theta(w)); }
__device__ __forceinline__ float tan_theta(f3 w) { return sin_theta(w) / w.y; }
__device__ __forceinline__ float tan2_theta(f3 w) { return sin2_theta(w) / cos2_theta(w); }
__device__ __forceinline__ float cos_phi(f3 w)
{
    const float st = sin_theta(w);
    return (st == 0.0f) ? 1.0f : std_clamp(w.x / st, -1.0f, 1.0f);
}
__device__ __forceinline__ float sin_phi(f3 w)
{
    const float st = sin_theta(w);
    return (st == 0.0f) ? 1.0f : std_clamp(w.z / st, -1.0f, 1.0f);
}
__device__ __forceinline__ bool same_hemisphere(f3 a, f3 b) { return a.y * b.y > 0.0f; }

// materials/Material.h:114
__device__ __forceinline__ float fresnel_dielectric(float cos_i, float eta_i, float eta_t)
{
    cos_i = std_clamp(cos_i, -1.0f, 1.0f);
    if (!(cos_i > 0.0f)) {
        const float s = eta_i; eta_i = eta_t; eta_t = s;
        cos_i = abs_f(cos_i);
    }
    const float sin_i = sqrt_unit(std_max(0.0f, 1.0f - cos_i * cos_i));
    const float sin_t = eta_i / eta_t * sin_i;
    if (sin_t >= 1) return 1.0f;
    const float cos_t = sqrt_unit(std_max(0.0f, 1.0f - sin_t * sin_t));
    const float parl  = ((eta_t * cos_i) - (eta_i * cos_t)) / ((eta_t * cos_i) + (eta_i * cos_t));
    const float perp  = ((eta_i * cos_i) - (eta_t * cos_t)) / ((eta_i * cos_i) + (eta_t * cos_t));
    return (parl * parl + perp * perp) / 2.0f;
}

// math/Math.h:230 erfinv
__device__ __forceinline__ float erfinv(float a)
{
    float       p;
    const float t = lm_logf(fma_f(a, 0.0f - a, 1.0f));
    if (abs_f(t) > 6.125f) {
        p = 3.03697567e-10f;
        p = fma_f(p, t, 2.93243101e-8f);
        p = fma_f(p, t, 1.22150334e-6f);
        p = fma_f(p, t, 2.84108955e-5f);
        p = fma_f(p, t, 3.93552968e-4f);
        p = fma_f(p, t, 3.02698812e-3f);
        p = fma_f(p, t, 4.83185798e-3f);
        p = fma_f(p, t, -2.64646143e-1f);
        p = fma_f(p, t, 8.40016484e-1f);
    } else {
        p = 5.43877832e-9f;
        p = fma_f(p, t, 1.43285448e-7f);
        p = fma_f(p, t, 1.22774793e-6f);
        p = fma_f(p, t, 1.12963626e-7f);
        p = fma_f(p, t, -5.61530760e-5f);
        p = fma_f(p, t, -1.47697632e-4f);
        p = fma_f(p, t, 2.31468678e-3f);
        p = fma_f(p, t, 1.15392581e-2f);
        p = fma_f(p, t, -2.32015476e-1f);
        p = fma_f(p, t, 8.86226892e-1f);
    }
    return a * p;
}

// materials/Material.cpp:14 beckmann_sample11
__device__ __forceinline__ P2 beckmann_sample11(float cos_theta_i, float U1, float U2)
{
    P2 s;
    if (cos_theta_i > .9999f) {
        const float r  = sqrt_f(-lm_logf(1.0f - U1));
        float       sp, cp;
        lm_sincosf_bounded(2.0f * k_pi * U2, &sp, &cp); // U2 in [0, 1): bounded argument
        s.x = r * cp;
        s.y = r * sp;
        return s;
    }
    const float sin_theta_i = sqrt_unit(std_max(0.0f, 1.0f - cos_theta_i * cos_theta_i));
    const float tan_theta_i = sin_theta_i / cos_theta_i;
    const float cot_theta_i = 1.0f / tan_theta_i;
    float       a           = -1.0f;
    float       c           = lm_erff(cot_theta_i);
    const float sample_x    = std_max(U1, 1e-6f);
    const float theta_i     = lm_acosf(cos_theta_i);
    const float fit         = 1.0f + theta_i * (-0.876f + theta_i * (0.4265f - 0.0594f * theta_i));
    float       b           = c - (1.0f + c) * lm_powf(1.0f - sample_x, fit);
    const float sqrt_pi_inv = 1.0f / sqrt_f(k_pi);
    const float normalization =
        1.0f / (1.0f + c + sqrt_pi_inv * tan_theta_i * lm_expf(-cot_theta_i * cot_theta_i));
#pragma unroll 1 // data-dependent exit: unrolled copies only grow the hot loop
    for (int it = 0; it < 9; ++it) {
        if (!(b >= a && b <= c)) b = 0.5f * (a + c);
        const float inv_erf = erfinv(b);
        const float value =
            normalization * (1.0f + b + sqrt_pi_inv * tan_theta_i * lm_expf(-inv_erf * inv_erf)) - sample_x;
        const float derivative = normalization * (1.0f - inv_erf * tan_theta_i);
        if (abs_f(value) < 1e-5f) break;
        if (value > 0) c = b;
        else a = b;
        b -= value / derivative;
    }
    s.x = erfinv(b);
    s.y = erfinv(2.0f * std_max(U2, 1e-6f) - 1.0f);
    return s;
}

// materials/Material.cpp:89 beckmann_sample
__device__ __forceinline__ f3 beckmann_sample(f3 wi, float ax, float ay, float U1, float U2, const Rsq& q)
{
    const f3 st = normalize(mk(ax * wi.x, wi.y, ay * wi.z), q);
    P2       sl = beckmann_sample11(st.y, U1, U2);
    const float tmp = cos_phi(st) * sl.x - sin_phi(st) * sl.y;
    sl.y            = sin_phi(st) * sl.x + cos_phi(st) * sl.y;
    sl.x            = tmp;
    sl.x            = ax * sl.x;
    sl.y            = ay * sl.y;
    return normalize(mk(-sl.x, 1.0f, -sl.y), q);
}

// BeckmannDistribution (materials/Material.h:213)
__device__ __forceinline__ float beck_D(const Material& m, f3 wh)
{
    const float t2 = tan2_theta(wh);
    if (__builtin_isinf(t2)) return 0.0f;
    const float c4 = cos2_theta(wh) * cos2_theta(wh);
    const float cp = cos_phi(wh), sp = sin_phi(wh);
    return lm_expf(-t2 * ((cp * cp) / (m.alpha_x * m.alpha_x) + (sp * sp) / (m.alpha_y * m.alpha_y))) /
           (k_pi * m.alpha_x * m.alpha_y * c4);
}
__device__ __forceinline__ float beck_lambda(const Material& m, f3 w)
{
    const float at = abs_f(tan_theta(w));
    if (__builtin_isinf(at)) return 0.0f;
    const float cp    = cos_phi(w), sp = sin_phi(w);
    const float alpha = sqrt_f((cp * cp) * (m.alpha_x * m.alpha_x) + (sp * sp) * (m.alpha_y * m.alpha_y));
    const float a     = 1.0f / (alpha * at);
    if (a >= 1.6f) return 0.0f;
    return (1.0f - 1.259f * a + 0.396f * (a * a)) / (3.535f * a + 2.181f * (a * a));
}
__device__ __forceinline__ float beck_G1(const Material& m, f3 w) { return 1.0f / (1.0f + beck_lambda(m, w)); }
__device__ __forceinline__ float beck_G(const Material& m, f3 wo, f3 wi) { return 1.0f / (1.0f + beck_lambda(m, wo) + beck_lambda(m, wi)); }
__device__ __forceinline__ float beck_pdf(const Material& m, f3 wo, f3 wh)
{
    if (m.sample_visible_area) return beck_D(m, wh) * beck_G1(m, wo) * abs_f(dot(wo, wh)) / abs_f(wo.y);
    return beck_D(m, wh) * abs_f(wh.y);
}
// materials/Material.cpp:111 (visible-area branch; the parser always builds it)
__device__ __forceinline__ f3 beck_sample_wh(const Material& m, f3 wo, Rng& rng, const Rsq& q)
{
    const bool flip = wo.y < 0.0f;
    // arguments evaluated right to left by GCC: U2 is drawn first
    const float U2 = next1D(rng);
    const float U1 = next1D(rng);
    f3 wh = beckmann_sample(flip ? neg(wo) : wo, m.alpha_x, m.alpha_y, U1, U2, q);
    if (flip) wh = neg(wh);
    return wh;
}

// MicrofacetReflection (materials/Material.h:386)
__device__ __forceinline__ rgb mf_eval(const Material& m, f3 wo, f3 wi, const Rsq& q)
{
    const float ao = abs_f(wo.y), ai = abs_f(wi.y);
    if (ai == 0.0f || ao == 0.0f) return mkc(0, 0, 0);
    f3 wh = add(wi, wo);
    if (wh.x == 0.0f && wh.y == 0.0f && wh.z == 0.0f) return mkc(0, 0, 0);
    wh            = normalize(wh, q);
    const float f = fresnel_dielectric(dot(wi, wh), 1.0f, m.microfacet_ior);
    return cdivs(cscale(cscale(cscale(m.microfacet_r, beck_D(m, wh)), beck_G(m, wo, wi)), f), 4.0f * ai * ao);
}
__device__ __forceinline__ float mf_pdf(const Material& m, f3 wo, f3 wi, const Rsq& q)
{
    if (!same_hemisphere(wo, wi)) return 0.0f;
    const f3 wh = normalize(add(wo, wi), q);
    return beck_pdf(m, wo, wh) / (4.0f * dot(wo, wh));
}
__device__ __forceinline__ MSample mf_sample(const Material& m, f3 wo, Rng& rng, const Rsq& q)
{
    MSample r;
    r.color = mkc(0, 0, 0);
    r.dir   = mk(0, 0, 0);
    r.pdf   = 0.0f;
    r.props = 0;
    if (wo.y == 0.0f) return r;
    const f3    wh = beck_sample_wh(m, wo, rng, q);
    const float dp = dot(wo, wh);
    if (dp < 0.0f) return r;
    // specular_reflection(wo, n) = -wo + 2 dot(wo,n) n
    const f3 wi = add(neg(wo), scale(2.0f * dot(wo, wh), wh));
    if (!same_hemisphere(wo, wi)) return r;
    r.pdf   = beck_pdf(m, wo, wh) / (4.0f * dp);
    r.color = mf_eval(m, wo, wi, q);
    r.dir   = wi;
    r.props = PROP_GLOSSY | PROP_REFLECTIVE;
    return r;
}
// BRDF::rho_impl default (materials/Material.h:299) for the microfacet lobe.  All 16 samples
// share wo, so everything beckmann_sample / beckmann_sample11 / the Smith lambda compute from wo
// alone is evaluated once (BeckPre) -- the same expressions on the same inputs, so every sample
// is bit-identical to mf_sample's; only the per-sample work (U1, U2 onwards) stays in the loop.
struct BeckPre {
    bool  flip, steep;
    f3    st;
    float cphi, sphi;
    float tan_theta_i, c0, fit, normalization, sqrt_pi_inv;
    float lam_wo;
};
__device__ __forceinline__ BeckPre beck_pre(const Material& m, f3 wo, const Rsq& q)
{
    BeckPre p;
    p.flip               = wo.y < 0.0f;
    const f3 wi          = p.flip ? neg(wo) : wo;
    p.st                 = normalize(mk(m.alpha_x * wi.x, wi.y, m.alpha_y * wi.z), q);
    p.cphi               = cos_phi(p.st);
    p.sphi               = sin_phi(p.st);
    const float cos_t    = p.st.y;
    p.steep              = cos_t > .9999f;
    p.tan_theta_i = p.c0 = p.fit = p.normalization = p.sqrt_pi_inv = 0.0f;
    if (!p.steep) {
        const float sin_theta_i = sqrt_unit(std_max(0.0f, 1.0f - cos_t * cos_t));
        p.tan_theta_i           = sin_theta_i / cos_t;
        const float cot_theta_i = 1.0f / p.tan_theta_i;
        p.c0                    = lm_erff(cot_theta_i);
        const float theta_i     = lm_acosf(cos_t);
        p.fit                   = 1.0f + theta_i * (-0.876f + theta_i * (0.4265f - 0.0594f * theta_i));
        p.sqrt_pi_inv           = 1.0f / sqrt_f(k_pi);
        p.normalization = 1.0f / (1.0f + p.c0 + p.sqrt_pi_inv * p.tan_theta_i * lm_expf(-cot_theta_i * cot_theta_i));
    }
    p.lam_wo = beck_lambda(m, wo);
    return p;
}
// beckmann_sample11 (materials/Material.cpp:14) from the precomputed wo terms
__device__ __forceinline__ P2 beckmann_sample11_pre(const BeckPre& p, float U1, float U2)
{
    P2 s;
    if (p.steep) {
        const float r  = sqrt_f(-lm_logf(1.0f - U1));
        float       sp, cp;
        lm_sincosf_bounded(2.0f * k_pi * U2, &sp, &cp); // U2 in [0, 1): bounded argument
        s.x = r * cp;
        s.y = r * sp;
        return s;
    }
    float       a        = -1.0f;
    float       c        = p.c0;
    const float sample_x = std_max(U1, 1e-6f);
    float       b        = c - (1.0f + c) * lm_powf(1.0f - sample_x, p.fit);
    // erfinv(b) at the converged b is the last iteration's inv_erf (same b, same function), so
    // the final erfinv is only evaluated when the loop ran out of iterations (b moved after it)
    float inv_erf   = 0.0f;
    bool  converged = false;
#if defined(SP_WAVE_PROF) && defined(SP_WPROF_NEWTON) // regions 4 / 5: each iteration / the whole loop
    const uint64_t t_nl = __builtin_amdgcn_s_memtime();
#endif
#pragma unroll 1 // data-dependent exit: unrolled copies only grow the hot loop
    for (int it = 0; it < 9; ++it) {
#if defined(SP_WAVE_PROF) && defined(SP_WPROF_NEWTON)
        const uint64_t t_it = __builtin_amdgcn_s_memtime();
#endif
        if (!(b >= a && b <= c)) b = 0.5f * (a + c);
        inv_erf = erfinv(b);
        const float value =
            p.normalization * (1.0f + b + p.sqrt_pi_inv * p.tan_theta_i * lm_expf(-inv_erf * inv_erf)) - sample_x;
        const float derivative = p.normalization * (1.0f - inv_erf * p.tan_theta_i);
#if defined(SP_WAVE_PROF) && defined(SP_WPROF_NEWTON)
        wprof_end(4, t_it);
#endif
        if (abs_f(value) < 1e-5f) {
            converged = true;
            break;
        }
        if (value > 0) c = b;
        else a = b;
        b -= value / derivative;
    }
#if defined(SP_WAVE_PROF) && defined(SP_WPROF_NEWTON)
    wprof_end(5, t_nl);
#endif
    s.x = converged ? inv_erf : erfinv(b);
    s.y = erfinv(2.0f * std_max(U2, 1e-6f) - 1.0f);
    return s;
}
__device__ __forceinline__ MSample mf_sample_pre_u(const Material& m, const BeckPre& p, f3 wo, uint64_t u2, uint64_t u1,
                                                   const Rsq& q);
// mf_sample with the precomputed wo terms (draw order: U2, then U1)
template <bool NT = false, bool PAIR = (SP_RNG_PAIR != 0)>
__device__ __forceinline__ MSample mf_sample_pre(const Material& m, const BeckPre& p, f3 wo, Rng& rng, const Rsq& q)
{
    MSample r;
    r.color = mkc(0, 0, 0);
    r.dir   = mk(0, 0, 0);
    r.pdf   = 0.0f;
    r.props = 0;
    if (wo.y == 0.0f) return r;
    uint64_t u2, u1;
    rng_raw2<NT, PAIR>(rng, u2, u1); // U2 first, then U1
    return mf_sample_pre_u(m, p, wo, u2, u1, q);
}
// mf_sample_pre_u's scalars: the sampled direction and pdf and the eval's factors, the microfacet
// colour left out (color = ((R * D) * G) * F / den per channel, 0 when black)
struct MGeom {
    f3    dir;
    float pdf; // 0: no sample (mf_sample_pre_u returns black, pdf 0)
    float D, G, F, den;
    bool  valid; // false: mf_sample_pre_u's early returns (black, no direction, pdf 0, no props)
    bool  black;
};
__device__ __forceinline__ MGeom mf_sample_geom(const Material& m, const BeckPre& p, f3 wo, uint64_t u2, uint64_t u1,
                                                const Rsq& q)
{
    MGeom g;
    g.dir   = mk(0, 0, 0);
    g.pdf   = 0.0f;
    g.D = g.G = g.F = 0.0f;
    g.den   = 1.0f;
    g.valid = false;
    g.black = true;
    const float U2 = canonical_from_u64(u2);
    const float U1 = canonical_from_u64(u1);
    P2          sl = beckmann_sample11_pre(p, U1, U2);
    const float tmp = p.cphi * sl.x - p.sphi * sl.y;
    sl.y            = p.sphi * sl.x + p.cphi * sl.y;
    sl.x            = tmp;
    sl.x            = m.alpha_x * sl.x;
    sl.y            = m.alpha_y * sl.y;
    f3 wh = normalize(mk(-sl.x, 1.0f, -sl.y), q);
    if (p.flip) wh = neg(wh);
    const float dp = dot(wo, wh);
    if (dp < 0.0f) return g;
    const f3 wi = add(neg(wo), scale(2.0f * dot(wo, wh), wh));
    if (!same_hemisphere(wo, wi)) return g;
    // beck_pdf(m, wo, wh) with G1(wo) = 1 / (1 + lambda(wo))
    const float bpdf = m.sample_visible_area ? beck_D(m, wh) * (1.0f / (1.0f + p.lam_wo)) * abs_f(dot(wo, wh)) / abs_f(wo.y)
                                             : beck_D(m, wh) * abs_f(wh.y);
    g.pdf   = bpdf / (4.0f * dp);
    g.dir   = wi;
    g.valid = true;
    // mf_eval(m, wo, wi) with G = 1 / (1 + lambda(wo) + lambda(wi))
    const float ao = abs_f(wo.y), ai = abs_f(wi.y);
    if (ai == 0.0f || ao == 0.0f) return g;
    f3 h = add(wi, wo);
    if (h.x == 0.0f && h.y == 0.0f && h.z == 0.0f) return g;
    h       = normalize(h, q);
    g.F     = fresnel_dielectric(dot(wi, h), 1.0f, m.microfacet_ior);
    g.G     = 1.0f / (1.0f + p.lam_wo + beck_lambda(m, wi));
    g.D     = beck_D(m, h);
    g.den   = 4.0f * ai * ao;
    g.black = false;
    return g;
}
// one channel of the sample's colour: cdivs(cscale(cscale(cscale(R, D), G), F), den) per channel
__device__ __forceinline__ float mf_geom_channel(const MGeom& g, float R) { return g.black ? 0.0f : (((R * g.D) * g.G) * g.F) / g.den; }
// mf_sample_pre from its two drawn (tempered) words
__device__ __forceinline__ MSample mf_sample_pre_u(const Material& m, const BeckPre& p, f3 wo, uint64_t u2, uint64_t u1,
                                                   const Rsq& q)
{
    const MGeom g = mf_sample_geom(m, p, wo, u2, u1, q);
    MSample     r;
    r.color = mkc(0, 0, 0);
    r.dir   = g.dir;
    r.pdf   = g.pdf;
    r.props = 0;
    if (!g.valid) return r;
    r.color = mkc(mf_geom_channel(g, m.microfacet_r.r), mf_geom_channel(g, m.microfacet_r.g), mf_geom_channel(g, m.microfacet_r.b));
    r.props = PROP_GLOSSY | PROP_REFLECTIVE;
    return r;
}
// The rho estimate's sum over one sample: r += color * |wi.y| / pdf per channel.  A grey microfacet
// colour (the three channels' bits equal: every glossy material a scene file makes has R = 1)
// computes one channel -- the other two would repeat its operations on the same bits.
__device__ __forceinline__ void rho_accumulate(rgb& r, const MGeom& g, rgb R, bool grey)
{
    if (!(g.pdf > 0.0f)) return;
    const float ay = abs_f(g.dir.y);
    r.r = r.r + (mf_geom_channel(g, R.r) * ay) / g.pdf;
    if (!grey) {
        r.g = r.g + (mf_geom_channel(g, R.g) * ay) / g.pdf;
        r.b = r.b + (mf_geom_channel(g, R.b) * ay) / g.pdf;
    }
}
// SP_RHO_ALIGNED: the estimate's 32 words (idx .. idx + 31, reserved: no twist) are read as one
// aligned 16-byte pair per sample, whatever the parity of idx: at an odd idx a sample's two words
// are the high word of one pair (carried from the previous load) and the low word of the next, so
// every lane runs the same code -- no branch between pair and single loads (rng_raw2), 16 loads
// per estimate.  Same words in the same order; the stream then skips the 32 words (the state 32
// draws leave).  Needs even lane blocks and no draw-ahead window.
#ifndef SP_RHO_ALIGNED
#define SP_RHO_ALIGNED 0
#endif
#ifndef SP_RHO_GREY // one channel of the rho estimate for a grey microfacet colour (rho_accumulate)
#define SP_RHO_GREY 1
#endif
template <bool PAIR = (SP_RNG_PAIR != 0), bool ALIGN = (SP_RHO_ALIGNED != 0), bool TOUCH = (SP_RHO_TOUCH != 0)>
__device__ __forceinline__ rgb mf_rho16(const Material& m, f3 wo, Rng& rng, const Rsq& q)
{
    const BeckPre p = beck_pre(m, wo, q);
    rgb           r = mkc(0, 0, 0);
    const bool grey = SP_RHO_GREY && f2u(m.microfacet_r.r) == f2u(m.microfacet_r.g) && f2u(m.microfacet_r.r) == f2u(m.microfacet_r.b);
    rng_reserve(rng, 32); // the loop below draws at most 32 words and never twists
#if SP_RHO_TOUCH
    if constexpr (TOUCH) rng_touch(rng, 32, (__attribute__((address_space(3))) void*)rho_rng_sink);
#endif
    if constexpr (ALIGN && MT_BLK % 2 == 0 && RNG_PF == 0 && !SP_XP_SERVED_FREE) {
        if (wo.y == 0.0f) return cdivs(r, (float)16u); // mf_sample draws nothing: every sample is black
        const int       odd   = rng.idx & 1;
        const uint64_t* cur   = mt_buf(rng, rng.cur);
        const uint64_t* next  = mt_buf(rng, mt_next(rng));
        uint64_t        carry = odd ? cur[mt_off(rng.idx)] : 0ull;
        for (unsigned i = 0; i < 16u; ++i) {
            const int       t = rng.idx + odd + 2 * (int)i; // even: a whole aligned pair
            const uint64_t* b = (t < MT_N) ? cur + mt_off(t) : next + mt_off(t - MT_N);
            SP_TD(td_lines(rng.td_cat, b, 16));
            const ulonglong2 w  = *reinterpret_cast<const ulonglong2*>(b);
            const uint64_t   w0 = odd ? carry : w.x, w1 = odd ? w.x : w.y;
            carry               = w.y;
            rho_accumulate(r, mf_sample_geom(m, p, wo, mt_temper(w0), mt_temper(w1), q), m.microfacet_r, grey);
        }
        rng_skip_reserved(rng, 32);
        if (grey) r.g = r.b = r.r;
        return cdivs(r, (float)16u);
    }
    for (unsigned i = 0; i < 16u; ++i) {
        if (wo.y == 0.0f) continue; // mf_sample_pre: draws nothing, black
        uint64_t u2, u1;
        rng_raw2<true, PAIR>(rng, u2, u1); // U2 first, then U1
        rho_accumulate(r, mf_sample_geom(m, p, wo, u2, u1, q), m.microfacet_r, grey);
    }
    if (grey) r.g = r.b = r.r;
    return cdivs(r, (float)16u);
}

#if SP_SERVE_RHO
// Per-wave LDS of the IterativeRRNEE megakernel, used by two phases of a bounce in turn:
//   serve_rho: srv_w [call site k][weight][owner lane] (weights served to the owners, 512 words)
//              and srv_req (request r: owner lane | k << 6, k = 3: the bounce's sample; 256 bytes);
//   the merged query pass (mq_run, after every served weight has been taken): the posted rays
//              and their results, MQ_* below.
#ifndef SP_MERGE_QUERIES
#define SP_MERGE_QUERIES 1
#endif
enum : int {
    MQ_O = 0,       // shared origin of an owner's two rays (x, y, z planes of 64)
    MQ_D3 = 192,    // MIS ray direction (estimate_direct_mis, Integrator.cpp:527-533)
    MQ_T3 = 384,    // its t_min
    MQ_D1 = 448,    // next bounce's direction (Integrator.cpp:570)
    MQ_T1 = 640,    // its t_min
    MQ_BEST = 704,  // next bounce's closest hit so far: u64 (t bits << 32 | wide slot) per owner
    MQ_ANY = 832,   // MIS ray's geometry any-hit result per owner
    MQ_TB = 896,    // per walking lane: pending stack entries [bot, top) and its query (thieves read it)
    MQ_Q = 960,     // queue: 128 bytes, query r = owner lane | any-hit << 7
    MQ_CNT = 992,   // next unclaimed query
    MQ_WORDS = 996, // a multiple of 4: every wave's row, and MQ_BEST's u64 slots, stay 16-byte aligned
    SRV_W = 0, SRV_REQ = 512, SRV_WORDS = 576,
    SRV_WAVE_WORDS = (SP_MERGE_QUERIES && MQ_WORDS > SRV_WORDS) ? MQ_WORDS : SRV_WORDS
};
static_assert(SRV_WAVE_WORDS % 4 == 0 && MQ_BEST % 2 == 0, "u64 LDS atomics need 8-byte alignment");
struct MqLayout { // IterativeRRNEE's rows for mq_run (the MIS / next-closest pass and the shadow pass)
    enum : int { O = MQ_O, D3 = MQ_D3, T3 = MQ_T3, D1 = MQ_D1, T1 = MQ_T1, BEST = MQ_BEST, AMAX = MQ_BEST, ANY = MQ_ANY,
                 TB = MQ_TB, Q = MQ_Q, CNT = MQ_CNT };
};
#ifndef SP_MQ_SHADOW // the shadow rays' walks shared too (mis_light_part_mq)
#define SP_MQ_SHADOW 1
#endif
static __shared__ __attribute__((aligned(16))) uint32_t srv_lds[4][SRV_WAVE_WORDS];
__device__ __forceinline__ float*   srv_w_at(int wave, int k, int j) { return reinterpret_cast<float*>(&srv_lds[wave][SRV_W + (k * 2 + j) * 64]); }
__device__ __forceinline__ uint8_t* srv_req_of(int wave) { return reinterpret_cast<uint8_t*>(&srv_lds[wave][SRV_REQ]); }
#endif

// OneSampleMaterial::get_selection_weights for the glossy pair {microfacet, lambertian}
template <bool PAIR = (SP_RNG_PAIR != 0), bool ALIGN = (SP_RHO_ALIGNED != 0), bool TOUCH = (SP_RHO_TOUCH != 0)>
__device__ __forceinline__ void glossy_weights(const Material& m, f3 wo, Rng& rng, const Rsq& q, float w[2])
{
#if SP_SERVE_RHO
    if (rng.srv_on == 1) {
        // the same estimate (same material, wo and stream words) was computed by the wave: take it
        // and advance the stream past its words
        const uint32_t d = rng.draws - rng.srv_pos;
        int            k = -1;
        if (rng.srv_A && rng.draws == rng.srv_posA) k = 3;
        else if (rng.srv_B) k = (d == 0u) ? 0 : (d == rng.srv_dc) ? 1 : (d == 2u * rng.srv_dc + rng.srv_coat) ? 2 : -1;
        if (k >= 0) {
            const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
            w[0]           = srv_w_at(wave, k, 0)[lane];
            w[1]           = srv_w_at(wave, k, 1)[lane];
            rng_skip_reserved(rng, (int)rng.srv_dc);
            return;
        }
    }
#endif
    rgb r0;
    SP_WPROF(1, r0 = (mf_rho16<PAIR, ALIGN, TOUCH>(m, wo, rng, q)));
    const rgb r1 = cscale(m.lambert_albedo, k_pi); // LambertianBRDF::rho_impl
    float     sum = 0.0f;
    w[0] = luminance(r0);
    sum += w[0];
    w[1] = luminance(r1);
    sum += w[1];
    w[0] = w[0] / sum;
    w[1] = w[1] / sum;
}
__device__ __forceinline__ float lambert_only_weight(const Material& m)
{
    const rgb r   = cscale(m.lambert_albedo, k_pi);
    float     sum = 0.0f;
    float     w   = luminance(r);
    sum += w;
    return w / sum;
}
__device__ __forceinline__ float balance(float p, float inner) { return (inner == 0.0f) ? 0.0f : p / inner; }

__device__ __forceinline__ MSample lambert_sample(const Material& m, Rng& rng)
{
    MSample r;
    const P2 u = next2D(rng);
    r.dir      = sample_uniform_hemisphere(u);
    r.color    = m.lambert_albedo;
    r.pdf      = k_uniform_hemisphere_pdf;
    r.props    = PROP_DIFFUSE | PROP_REFLECTIVE;
    return r;
}

// Local-space sample/eval/pdf of a non-clearcoat material (OneSampleMaterial).  The glossy forms
// are split at the selection-weight estimate: *_w take the weights glossy_weights produced.
__device__ __forceinline__ MSample onesample_sample_w(const Material& m, f3 wo, const float w[2], Rng& rng, const Rsq& q)
{
    const float u   = next1D(rng);
    float       cdf = 0.0f;
    int         sel = 1; // loop falls through only on NaN weights (uninitialised in the reference)
    for (int i = 0; i < 2; ++i) {
        if (w[i] + cdf > u) { sel = i; break; }
        cdf += w[i];
    }
    MSample res = (sel == 0) ? mf_sample(m, wo, rng, q) : lambert_sample(m, rng);
    if (res.pdf == 0.0f || cblack(res.color)) {
        MSample z;
        z.color = mkc(0, 0, 0); z.dir = mk(0, 0, 0); z.pdf = 0.0f; z.props = 0;
        return z;
    }
    const f3 wi = res.dir;
    rgb      values[2];
    float    pdfs[2];
    for (int i = 0; i < 2; ++i) {
        if (i == sel) {
            values[i] = res.color;
            pdfs[i]   = res.pdf * w[i];
        } else if (i == 0) {
            values[i] = mf_eval(m, wo, wi, q);
            pdfs[i]   = mf_pdf(m, wo, wi, q) * w[i];
        } else {
            values[i] = m.lambert_albedo;
            pdfs[i]   = k_uniform_hemisphere_pdf * w[i];
        }
    }
    const float inner = (0.0f + pdfs[0]) + pdfs[1];
    rgb         col   = mkc(0, 0, 0);
    float       pdf   = 0.0f;
    for (int i = 0; i < 2; ++i) {
        if (pdfs[i] > 0.0f) {
            const float mw = balance(pdfs[i], inner);
            col            = cadd(col, cscale(values[i], mw));
            pdf += pdfs[i];
        }
    }
    MSample out;
    out.color = col;
    out.dir   = wi;
    out.pdf   = pdf;
    out.props = res.props;
    return out;
}
__device__ __forceinline__ MSample onesample_sample(const Material& m, f3 wo, Rng& rng, const Rsq& q)
{
    if (m.kind == SP_MAT_LAMBERTIAN) return lambert_sample(m, rng);
    float w[2];
    glossy_weights(m, wo, rng, q, w);
    return onesample_sample_w(m, wo, w, rng, q);
}

__device__ __forceinline__ rgb onesample_eval_w(const Material& m, f3 wo, f3 wi, const float w[2], const Rsq& q)
{
    const float p0    = mf_pdf(m, wo, wi, q) * w[0];
    const float p1    = k_uniform_hemisphere_pdf * w[1];
    const float inner = (0.0f + p0) + p1;
    rgb         r     = mkc(0, 0, 0);
    if (p0 > 0.0f) r = cadd(r, cscale(mf_eval(m, wo, wi, q), balance(p0, inner)));
    if (p1 > 0.0f) r = cadd(r, cscale(m.lambert_albedo, balance(p1, inner)));
    return r;
}
__device__ __forceinline__ rgb onesample_eval(const Material& m, f3 wo, f3 wi, Rng& rng, const Rsq& q)
{
    if (m.kind == SP_MAT_LAMBERTIAN) {
        const float w     = lambert_only_weight(m);
        const float p     = k_uniform_hemisphere_pdf * w;
        const float inner = 0.0f + p;
        rgb         r     = mkc(0, 0, 0);
        if (p > 0.0f) r = cadd(r, cscale(m.lambert_albedo, balance(p, inner)));
        return r;
    }
    float w[2];
    glossy_weights(m, wo, rng, q, w);
    return onesample_eval_w(m, wo, wi, w, q);
}

__device__ __forceinline__ float onesample_pdf_w(const Material& m, f3 wo, f3 wi, const float w[2], const Rsq& q)
{
    float p = 0.0f;
    p += w[0] * mf_pdf(m, wo, wi, q);
    p += w[1] * k_uniform_hemisphere_pdf;
    return p;
}
__device__ __forceinline__ float onesample_pdf(const Material& m, f3 wo, f3 wi, Rng& rng, const Rsq& q)
{
    if (m.kind == SP_MAT_LAMBERTIAN) {
        const float w = lambert_only_weight(m);
        float       p = 0.0f;
        p += w * k_uniform_hemisphere_pdf;
        return p;
    }
    float w[2];
    glossy_weights(m, wo, rng, q, w);
    return onesample_pdf_w(m, wo, wi, w, q);
}

// Material::sample/eval/pdf incl. ClearcoatMaterial (materials/Material.h:461-529, 723-806)
// Does Material::eval / sample / pdf at this record run the 16-sample glossy estimate?
__device__ __forceinline__ bool material_has_rho(const Scene& sc, int mid)
{
    const Material& m = sc.materials[mid];
    const int       k = (m.kind == SP_MAT_CLEARCOAT) ? sc.materials[m.base].kind : m.kind;
    return k == SP_MAT_GLOSSY;
}

// A clearcoat's base and a plain material share ONE inlined copy of the OneSample code (the
// 16-sample glossy estimate is ~5 K instructions): the coat only selects which record that copy
// reads and wraps its result.  Two copies measured as two hot loops competing for the
// instruction cache.  The coat's Fresnel term draws nothing, so computing it before or after the
// base changes no value.
__device__ __forceinline__ MSample material_sample_local(const Scene& sc, int mid, f3 wo, Rng& rng, const Rsq& q)
{
    const Material& m    = sc.materials[mid];
    const bool      coat = m.kind == SP_MAT_CLEARCOAT;
    float           f    = 0.0f;
    if (coat) {
        f             = fresnel_dielectric(wo.y, 1.0f, m.coat_ior);
        const float u = next1D(rng);
        if (u < f) {
            MSample s;
            s.dir   = mk(-wo.x, wo.y, -wo.z);
            s.color = cdivs(cscale(m.coat_color, f), abs_f(s.dir.y));
            s.pdf   = f;
            s.props = PROP_SPECULAR | PROP_REFLECTIVE;
            return s;
        }
    }
    const MSample b = onesample_sample(sc.materials[coat ? m.base : mid], wo, rng, q);
    if (!coat || b.pdf == 0.0f) return b;
    MSample s;
    s.pdf   = (1.0f - f) * b.pdf;
    s.color = cmul(csub(mkc(1, 1, 1), cscale(m.coat_color, f)), b.color);
    s.dir   = b.dir;
    s.props = b.props;
    return s;
}
__device__ __forceinline__ rgb material_eval_local(const Scene& sc, int mid, f3 wo, f3 wi, Rng& rng, const Rsq& q)
{
    const Material& m    = sc.materials[mid];
    const bool      coat = m.kind == SP_MAT_CLEARCOAT;
    const rgb       r    = onesample_eval(sc.materials[coat ? m.base : mid], wo, wi, rng, q);
    if (!coat) return r;
    const float f = fresnel_dielectric(wo.y, 1.0f, m.coat_ior);
    return cscale(r, 1.0f - f);
}
__device__ __forceinline__ float material_pdf_local(const Scene& sc, int mid, f3 wo, f3 wi, Rng& rng, const Rsq& q)
{
    const Material& m    = sc.materials[mid];
    const bool      coat = m.kind == SP_MAT_CLEARCOAT;
    const float     p    = onesample_pdf(sc.materials[coat ? m.base : mid], wo, wi, rng, q);
    if (!coat) return p;
    const float f = fresnel_dielectric(wo.y, 1.0f, m.coat_ior);
    return (1.0f - f) * p;
}

__device__ __forceinline__ MSample material_sample(const Scene& sc, int mid, f3 wo_w, f3 n, Rng& rng, const Rsq& q)
{
    const Onb o = onb_from_v(n, q);
    MSample   r = material_sample_local(sc, mid, to_onb(o, wo_w), rng, q);
    if (r.pdf == 0.0f || cblack(r.color)) return r;
    r.dir = to_world(o, r.dir);
    return r;
}
__device__ __forceinline__ rgb material_eval(const Scene& sc, int mid, f3 wo, f3 wi, f3 n, Rng& rng, const Rsq& q)
{
    const Onb o = onb_from_v(n, q);
    return material_eval_local(sc, mid, to_onb(o, wo), to_onb(o, wi), rng, q);
}
__device__ __forceinline__ float material_pdf(const Scene& sc, int mid, f3 wo, f3 wi, f3 n, Rng& rng, const Rsq& q)
{
    const Onb o = onb_from_v(n, q);
    return material_pdf_local(sc, mid, to_onb(o, wo), to_onb(o, wi), rng, q);
}

// ------------------------------------------------------------------------------ light sampling
struct LSample {
    rgb   L;
    float pdf;
    Ray   ray;
    float tmin, tmax;
};

// Sphere::pdf (shapes/Sphere.h:271)
__device__ __forceinline__ float sphere_pdf(const Light& l, f3 observer_world)
{
    const f3    obs = xfm_point(l.w2o, observer_world);
    const float sqr = dot(obs, obs);
    if (sqr <= 1.0f) return k_uniform_sphere_pdf;
    constexpr float sin2_1_5_deg = 0.00068523f;
    const float     sin2_max     = 1.0f / sqr;
    const float     cos_max      = sqrt_unit(std_max(0.0f, 1.0f - sin2_max));
    const float     omc          = (sin2_max < sin2_1_5_deg) ? sin2_max / 2.0f : 1.0f - cos_max;
    return 1.0f / (2.0f * k_pi * omc);
}

// Light::sample (Lights/Light.h:145) for SphereLight / EnvironmentLight / ImageBasedEnvironmentLight
__device__ __forceinline__ LSample light_sample(const Scene& sc, const Light& l, f3 obs, f3 obs_n, P2 u, const Rsq& q)
{
    LSample s;
    f3      wi;
    float   pdf, max_dist;
    s.L = l.radiance;
    if (l.kind == SP_LIGHT_SPHERE) {
        // Sphere::sample(observer, u) (shapes/Sphere.h:245)
        const f3 lo = xfm_point(l.w2o, obs);
        f3       local;
        if (dot(lo, lo) <= 1.0f) {
            local = sample_uniform_sphere(u);
        } else {
            const f3  smp = sample_cosine_hemisphere(u);
            const Onb o   = onb_from_v(lo, q);
            local         = to_world(o, smp);
        }
        const f3 sp_w = xfm_point(l.o2w, local);
        const f3 sn_w = xfm_vector(l.nrm, local);
        // ObjectLight::sample_impl (Lights/Light.h:188)
        const f3 to_sample = sub(sp_w, obs);
        wi                 = normalize(to_sample, q);
        pdf                = sphere_pdf(l, obs);
        max_dist           = length(to_sample) - ray_offset(sn_w, neg(wi));
    } else if (l.kind == SP_LIGHT_IMAGE_ENVIRONMENT) {
        const EnvSample es = env_sample(sc.envs[l.image], u);
        wi                 = es.wi;
        pdf                = es.pdf;
        s.L                = es.L;
        max_dist           = k_infinite;
    } else {
        // EnvironmentLight::light_sample (Lights/Light.h:265)
        wi       = sample_uniform_sphere(u);
        pdf      = k_uniform_sphere_pdf;
        max_dist = k_infinite;
    }
    s.pdf   = pdf;
    s.tmin  = ray_offset(obs_n, wi);
    s.tmax  = max_dist;
    s.ray.o = obs;
    s.ray.d = wi;
    return s;
}
// Light::pdf (Lights/Light.h:54)
__device__ __forceinline__ float light_pdf(const Scene& sc, const Light& l, f3 obs, f3 wi)
{
    if (l.kind == SP_LIGHT_SPHERE) return sphere_pdf(l, obs);
    if (l.kind == SP_LIGHT_IMAGE_ENVIRONMENT) return env_pdf(sc.envs[l.image], wi);
    return k_uniform_sphere_pdf;
}

// ============================================================================ integrators
#ifndef SP_OCC_CACHE // round 5 default 1; level on every config (profiles/r05/walk_cache/), off since round 6 (wide_any)
#define SP_OCC_CACHE 0
#endif
struct Ctx {
    const Scene& sc;
    Rng&         rng;
    const Rsq&   q;
    Stack        st;
    uint32_t     rays, shadow;
    // occluder cache (SP_OCC_CACHE): the wide slot of this lane's last occluder, tried first by the
    // next shadow walk; a pixel's samples run on one lane, so the previous sample's occluder is the
    // likeliest (~0: none).  Level on bunny / lucy / the shards, where it applies;
    // the same cache for closest hits (the previous hit tested first) lost 1 % on lucy.
    uint32_t     occ_slot = 0xffffffffu;
    // recursive integrators with max_depth > MAX_RECURSION: per-level records in global memory,
    // record k of this lane at deep[k * dstride] (level-major, lanes contiguous)
    float*       deep    = nullptr;
    size_t       dstride = 0;
#ifdef SP_MEGA_PROF // diagnostic build: shader clocks spent in trace / light sample / eval / occlusion
    uint64_t prof[4] = { 0, 0, 0, 0 };
#endif
};
#ifdef SP_MEGA_PROF
#define SP_PROF(k, stmt)                                                                                               \
    do {                                                                                                               \
        const uint64_t t_prof_ = __builtin_amdgcn_s_memtime();                                                         \
        stmt;                                                                                                          \
        c.prof[k] += __builtin_amdgcn_s_memtime() - t_prof_;                                                           \
    } while (0)
#else
#define SP_PROF(k, stmt) stmt
#endif

__device__ __forceinline__ bool occluded(Ctx& c, const Ray& r, float tmin, float tmax)
{
    ++c.shadow;
    ++c.rays;
    bool hit;
    SP_WPROF(3, hit = scene_any(c.sc, r, tmin, tmax, c.st, SP_OCC_CACHE ? &c.occ_slot : nullptr));
    return hit;
}

// Shared "primary" query of every integrator: intersect_lights then intersect.
struct Query {
    LightHit lh;
    bool     geom;
    Isect    is;
};
__device__ __forceinline__ Query trace(Ctx& c, const Ray& ray, float tmin, float tmax)
{
    Query qr;
    ++c.rays;
    Hit h;
    SP_WPROF(2, {
        qr.lh = scene_intersect_lights(c.sc, ray, tmin, tmax, c.st);
        if (qr.lh.hit) tmax = qr.lh.t;
        h = scene_intersect(c.sc, ray, tmin, tmax, c.st);
    });
    qr.geom     = (h.code != 0xffffffffu);
    if (qr.geom) qr.is = finish_hit(c.sc, h, ray, c.q);
    return qr;
}

// DirectLightingIntegrator::do_integrate (Integrators/Integrator.cpp:277) -- also the NEE part
// of WhittedIntegrator.
__device__ __forceinline__ rgb direct_nee(Ctx& c, const Isect& is, f3 wo)
{
    rgb L = mkc(0, 0, 0);
    for (int li = 0; li < c.sc.n_lights; ++li) {
        const Light l = uload_light(c.sc.lights + li);
        LSample     ls;
        SP_PROF(1, ls = light_sample(c.sc, l, is.p, is.n, next2D(c.rng), c.q));
        if (ls.pdf == 0.0f || cblack(ls.L)) continue;
        const f3 wi = ls.ray.d;
        rgb      f;
        SP_PROF(2, f = material_eval(c.sc, is.material, wo, wi, is.n, c.rng, c.q));
        bool vis = false;
        if (!cblack(f)) SP_PROF(3, vis = !occluded(c, ls.ray, ls.tmin, ls.tmax));
        if (vis) L = cadd(L, cdivs(cscale(cmul(f, ls.L), abs_f(dot(wi, is.n))), ls.pdf));
    }
    return L;
}

// Stream words one direct_nee call at hit `is` draws: two per light for Light::sample, plus 32
// for the glossy rho estimate of Material::eval when the light sample is usable and wo.y != 0 in
// the shading frame.  For sphere and uniform environment lights usability (pdf != 0, L not black)
// does not depend on the drawn numbers -- pdf is sphere_pdf(observer) or a constant, L the
// radiance -- so the count is known from the hit (the sample chunks, sp_chunk.hip, and the
// megakernel's tail chunks, sp_mega.hpp; not used with an image light).
__device__ __forceinline__ uint32_t sample_draws(const Scene& sc, const Isect& is, f3 wo, const Rsq& q)
{
    const Material& m    = sc.materials[is.material];
    const int       base = (m.kind == SP_MAT_CLEARCOAT) ? sc.materials[m.base].kind : m.kind;
    bool            rho  = false;
    if (base != SP_MAT_LAMBERTIAN) {
        const Onb o = onb_from_v(is.n, q);
        rho         = to_onb(o, wo).y != 0.0f;
    }
    uint32_t n = 0;
    for (int li = 0; li < sc.n_lights; ++li) {
        const Light lt  = uload_light(sc.lights + li);
        const float pdf = (lt.kind == SP_LIGHT_SPHERE) ? sphere_pdf(lt, is.p) : k_uniform_sphere_pdf;
        n += 2;
        if (rho && !(pdf == 0.0f || cblack(lt.radiance))) n += 32;
    }
    return n;
}

__device__ __forceinline__ rgb integrate_direct(Ctx& c, Ray ray)
{
    rgb L = mkc(0, 0, 0);
    if (0 >= c.sc.max_depth) return L;
    Query qr;
    SP_PROF(0, qr = trace(c, ray, k_ray_epsilon, k_infinite));
    if (qr.geom) {
        L = direct_nee(c, qr.is, neg(ray.d));
    } else if (qr.lh.hit) {
        L = cadd(L, cmul(mkc(1, 1, 1), light_hit_L(c.sc, qr.lh, ray.d, c.q)));
    }
    return L;
}

// BruteForceIntegratorIterative(RR) (Integrators/Integrator.cpp:160 / 211)
template <bool RR>
__device__ __forceinline__ rgb integrate_iterative(Ctx& c, Ray ray)
{
    rgb   throughput = mkc(1, 1, 1);
    rgb   L          = mkc(0, 0, 0);
    float tmin = k_ray_epsilon, tmax = k_infinite;
    constexpr float rr_cut = 0.1f;
    for (int depth = 0; depth < c.sc.max_depth; ++depth) {
        rng_prepare(c.rng);
        const Query qr = trace(c, ray, tmin, tmax);
        if (qr.geom) {
            const f3      wo = neg(ray.d);
            const f3      n  = qr.is.n;
            const MSample s  = material_sample(c.sc, qr.is.material, wo, n, c.rng, c.q);
            if (s.pdf == 0.0f || cblack(s.color)) break;
            const f3    wi     = s.dir;
            const float cosine = abs_f(dot(wi, n));
            throughput         = cmul(throughput, cdivs(cscale(s.color, cosine), s.pdf));
            if (RR && depth >= c.sc.rr_depth) {
                const float lum = luminance(throughput);
                if (lum < rr_cut) {
                    const float qv = std_max(0.05f, lum / rr_cut);
                    if (next1D(c.rng) < qv) throughput = cdivs(throughput, qv);
                    else break;
                }
            }
            ray.o = ray_at(ray, qr.is.t);
            ray.d = wi;
            tmin  = ray_offset(cosine);
            tmax  = k_infinite;
        } else if (qr.lh.hit) {
            L = cadd(L, cmul(throughput, light_hit_L(c.sc, qr.lh, ray.d, c.q)));
            break;
        } else {
            break;
        }
    }
    return L;
}

// BruteForceIntegrator (recursive, Integrators/Integrator.cpp:116), unrolled: the recursion's
// product ((L_{k+1} * cos_k) * color_k) / pdf_k is folded back from the deepest level.
constexpr int MAX_RECURSION = 32;
__device__ __forceinline__ rgb integrate_bruteforce(Ctx& c, Ray ray)
{
    float cosv[MAX_RECURSION];
    rgb   colv[MAX_RECURSION];
    float pdfv[MAX_RECURSION];
    int   depth = 0;
    rgb   Lend  = mkc(0, 0, 0);
    // levels beyond the register/scratch arrays go to the lane's global records (5 floats each)
    const bool deep = c.deep != nullptr;
    const int  maxd = deep ? c.sc.max_depth : (c.sc.max_depth < MAX_RECURSION ? c.sc.max_depth : MAX_RECURSION);
    auto put = [&](int k, float cs, rgb col, float pdf) {
        if (!deep) { cosv[k] = cs; colv[k] = col; pdfv[k] = pdf; return; }
        float* d = c.deep + (size_t)k * 5 * c.dstride;
        d[0] = cs; d[c.dstride] = col.r; d[2 * c.dstride] = col.g; d[3 * c.dstride] = col.b; d[4 * c.dstride] = pdf;
    };
    while (true) {
        if (depth >= maxd) { Lend = mkc(0, 0, 0); break; }
        rng_prepare(c.rng);
        const Query qr = trace(c, ray, k_ray_epsilon, k_infinite);
        if (qr.geom) {
            const f3      wo = neg(ray.d);
            const f3      n  = qr.is.n;
            const MSample s  = material_sample(c.sc, qr.is.material, wo, n, c.rng, c.q);
            if (s.pdf == 0.0f || cblack(s.color)) { Lend = mkc(0, 0, 0); break; }
            put(depth, dot(s.dir, n), s.color, s.pdf);
            ray.o       = ray_at(ray, qr.is.t);
            ray.d       = s.dir;
            ++depth;
        } else if (qr.lh.hit) {
            Lend = light_hit_L(c.sc, qr.lh, ray.d, c.q);
            break;
        } else {
            Lend = mkc(0, 0, 0);
            break;
        }
    }
    for (int k = depth - 1; k >= 0; --k) {
        float cs, pdf;
        rgb   col;
        if (!deep) { cs = cosv[k]; col = colv[k]; pdf = pdfv[k]; }
        else {
            const float* d = c.deep + (size_t)k * 5 * c.dstride;
            cs = d[0]; col = mkc(d[c.dstride], d[2 * c.dstride], d[3 * c.dstride]); pdf = d[4 * c.dstride];
        }
        Lend = cdivs(cmul(cscale(Lend, cs), col), pdf);
    }
    return Lend;
}

// WhittedIntegrator (Integrators/Integrator.cpp:323): NEE at every hit, recursion on specular.
// L_k += do_integrate(child) folds right-nested: L_0 + (L_1 + (L_2 + ...)).
__device__ __forceinline__ rgb integrate_whitted(Ctx& c, Ray ray)
{
    rgb        Lv[MAX_RECURSION + 1];
    int        depth = 0;
    const bool deep  = c.deep != nullptr; // levels in the lane's global records (3 floats each)
    const int  maxd  = deep ? c.sc.max_depth : (c.sc.max_depth < MAX_RECURSION ? c.sc.max_depth : MAX_RECURSION);
    auto put = [&](int k, rgb L) {
        if (!deep) { Lv[k] = L; return; }
        float* d = c.deep + (size_t)k * 3 * c.dstride;
        d[0] = L.r; d[c.dstride] = L.g; d[2 * c.dstride] = L.b;
    };
    auto get = [&](int k) {
        if (!deep) return Lv[k];
        const float* d = c.deep + (size_t)k * 3 * c.dstride;
        return mkc(d[0], d[c.dstride], d[2 * c.dstride]);
    };
    while (true) {
        rgb L = mkc(0, 0, 0);
        if (depth >= maxd) { put(depth, L); break; }
        rng_prepare(c.rng);
        const Query qr   = trace(c, ray, k_ray_epsilon, k_infinite);
        bool        more = false;
        if (qr.geom) {
            const f3 wo = neg(ray.d);
            L           = direct_nee(c, qr.is, wo);
            if (depth < c.sc.max_depth) {
                const MSample s = material_sample(c.sc, qr.is.material, wo, qr.is.n, c.rng, c.q);
                if (s.props & PROP_SPECULAR) {
                    ray.o = qr.is.p;
                    ray.d = s.dir;
                    more  = true;
                }
            }
        } else if (qr.lh.hit) {
            L = cadd(L, cmul(mkc(1, 1, 1), light_hit_L(c.sc, qr.lh, ray.d, c.q)));
        }
        put(depth, L);
        if (!more) break;
        ++depth;
    }
    rgb acc = get(depth);
    for (int k = depth - 1; k >= 0; --k) acc = cadd(get(k), acc);
    return acc;
}

// estimate_direct_mis (Integrators/Integrator.cpp:486), in two parts: the light sample and its
// shadow ray (true: the light sample is usable and unoccluded), then the rest
__device__ __forceinline__ bool mis_light_part(Ctx& c, const Light& l, f3 p, f3 n, LSample& ls)
{
    ls = light_sample(c.sc, l, p, n, next2D(c.rng), c.q);
    if (ls.pdf == 0.0f || cblack(ls.L)) return false;
    if (occluded(c, ls.ray, ls.tmin, ls.tmax)) return false;
    return true;
}
__device__ __forceinline__ rgb mis_material_part(Ctx& c, const Light& l, const LSample& ls, f3 p, f3 n, f3 wo, int mid)
{
    rgb       Lr = mkc(0, 0, 0);
    const f3  wi = ls.ray.d;
    const rgb be = material_eval(c.sc, mid, wo, wi, n, c.rng, c.q);
    if (!cblack(be)) {
        const float bp = material_pdf(c.sc, mid, wo, wi, n, c.rng, c.q);
        if (bp > 0.0f) {
            const float w = balance(ls.pdf, ls.pdf + bp);
            Lr            = cadd(Lr, cscale(cmul(be, ls.L), abs_f(dot(wi, n)) * w / ls.pdf));
        }
    }
    const MSample ms = material_sample(c.sc, mid, wo, n, c.rng, c.q);
    if (ms.pdf == 0.0f || cblack(ms.color)) return Lr;
    const float lp = light_pdf(c.sc, l, p, ms.dir);
    if (lp == 0.0f) return Lr;
    const float w = balance(ms.pdf, ms.pdf + lp);
    Ray         mr;
    mr.o             = p;
    mr.d             = ms.dir;
    const float mmin = ray_offset(n, ms.dir);
    ++c.rays;
    LightHit lh;
    SP_WPROF(3, lh = scene_intersect_lights(c.sc, mr, mmin, k_infinite, c.st));
    if (lh.hit) {
        if (!occluded(c, mr, mmin, k_infinite))
            Lr = cadd(Lr, cdivs(cscale(cscale(cmul(ms.color, light_hit_L(c.sc, lh, mr.d, c.q)), abs_f(dot(ms.dir, n))), w), ms.pdf));
    }
    return Lr;
}
__device__ __forceinline__ rgb estimate_direct_mis(Ctx& c, const Light& l, f3 p, f3 n, f3 wo, int mid)
{
    LSample ls;
    if (!mis_light_part(c, l, p, n, ls)) return mkc(0, 0, 0);
    return mis_material_part(c, l, ls, p, n, wo, mid);
}

#if SP_SERVE_RHO
// Wave-served selection-weight estimates (IterativeRRNEE).  After its shadow ray, a lane whose
// light sample is usable and unoccluded runs the glossy 16-sample estimate at three call sites
// in a row -- Material::eval, Material::pdf, Material::sample (Integrator.cpp:505-519) -- all with
// the same material and wo, at stream positions that are known in advance: eval's estimate takes
// the next 32 words (none when wo.y == 0), pdf's the 32 after them, and sample's starts one word
// later for a clearcoat (its Fresnel draw).  In lock step each call site costs the wave a full
// estimate however few lanes reach it.  Here the wave lists every such lane's three estimates,
// deals them out to all 64 lanes (dead paths and occluded lanes included), and each lane computes
// the estimates it is dealt from the owner's own stream words, read where the owner's state lives
// (the owner reserved the next generation first, so no twist happens in between).  The owners
// then take the weights at their call sites (glossy_weights) and skip the words.  Every estimate
// is the same function of the same inputs, so images, ray and draw counts are bit-identical.
// The sample call site's estimate is speculative: it is unused if the coat draw picks the
// specular lobe, and if eval's result is black (pdf's estimate then does not run) its position
// does not match and the owner computes it itself.
// One served estimate: glossy_weights at word idx of generation buffer cur of the owner's stream
// (reserved by the owner).  Inlined: 744-747 against 736-743 Mrays/s as a called function (elf
// 1024^2 @ 16 spp, profiles/r03/ab_rrnee_served.txt).
__device__ __forceinline__ void served_weights(const Material& m, f3 wo, uint64_t* base, int cur, int idx, const Rsq& q,
                                               float w[2])
{
    Rng sr;
    SP_TD(sr.td_cat = TD_SERVED);
    sr.base  = base;
    sr.cur   = cur;
    sr.idx   = idx;
    sr.ready = 1;
    sr.draws = 0;
    if (SP_XP_SERVED_FREE) sr.lin = 2;
    glossy_weights<(SP_SERVED_PAIR != 0), (SP_SERVED_ALIGNED != 0), (SP_SERVED_TOUCH != 0)>(m, wo, sr, q, w);
}
// want: this lane's eval / pdf / sample estimates of the light being estimated (k = 0, 1, 2);
// want_a: its deferred Material::sample of the bounce (k = 3, at c.rng.srv_pwA).  All lanes call.
__device__ __forceinline__ void serve_rho(Ctx& c, bool want, bool want_a, int mid, f3 n, f3 wo)
{
    const uint64_t mb = __ballot(want), ma = __ballot(want_a);
    if ((mb | ma) == 0) return;
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    f3        wl   = mk(0, 0, 0);
    int       base = 0;
    uint32_t  dc = 0, coat = 0, pw = 0, pwa = 0;
    if (want || want_a) {
        const Material& mm = c.sc.materials[mid];
        coat               = (mm.kind == SP_MAT_CLEARCOAT) ? 1u : 0u;
        base               = coat ? mm.base : mid;
        wl                 = to_onb(onb_from_v(n, c.q), wo); // the wo every call site passes on
        dc                 = (wl.y == 0.0f) ? 0u : 32u;      // mf_sample draws nothing when wo.y == 0
        const uint64_t lt  = (1ull << lane) - 1ull;
        int            r   = 3 * __popcll(mb & lt) + __popcll(ma & lt);
        if (want) {
            rng_reserve(c.rng, (int)(3u * dc + coat));
            pw = ((uint32_t)c.rng.cur << 16) | (uint32_t)c.rng.idx;
            for (int k = 0; k < 3; ++k) srv_req_of(wave)[r++] = (uint8_t)(lane | (k << 6));
            c.rng.srv_on   = 1;
            c.rng.srv_B    = true;
            c.rng.srv_pos  = c.rng.draws;
            c.rng.srv_dc   = dc;
            c.rng.srv_coat = coat;
        }
        if (want_a) {
            pwa                 = c.rng.srv_pwA;
            srv_req_of(wave)[r++] = (uint8_t)(lane | (3 << 6));
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const int total = 3 * __popcll(mb) + __popcll(ma);
    // requests are dealt to the lanes that are here: on a clipped border tile the pixels outside
    // the image never enter integrate(), so lane ids are not request slots -- rank the active lanes
    const uint64_t act  = __ballot(1);
    const int      rank = __popcll(act & ((1ull << lane) - 1ull));
    const int      nact = __popcll(act);
    for (int r0 = 0; r0 < total; r0 += nact) {
        const int      r = r0 + rank;
        const uint32_t e = (r < total) ? (uint32_t)srv_req_of(wave)[r] : 0u;
        const int      o = (int)(e & 63u), k = (int)(e >> 6);
        // the owner's inputs (all lanes take part in the exchange)
        const f3       owo   = mk(__shfl(wl.x, o, 64), __shfl(wl.y, o, 64), __shfl(wl.z, o, 64));
        const int      obase = __shfl(base, o, 64);
        const uint32_t opb   = (uint32_t)__shfl((int)pw, o, 64);
        const uint32_t opa   = (uint32_t)__shfl((int)pwa, o, 64);
        const uint32_t opw   = (k == 3) ? opa : opb;
        const uint32_t odc   = (uint32_t)__shfl((int)dc, o, 64);
        const uint32_t ocoat = (uint32_t)__shfl((int)coat, o, 64);
        if (r < total) {
            int cur = (int)(opw >> 16);
            int idx = (int)(opw & 0xffffu) + (int)(k == 0 || k == 3 ? 0u : k == 1 ? odc : 2u * odc + ocoat);
            if (idx >= MT_N) {
                cur ^= 1; // the megakernel's two-generation ring
                idx -= MT_N;
            }
            float w[2];
            served_weights(c.sc.materials[obase], owo, c.rng.base + (o - lane) * MT_BLK, cur, idx, c.q, w);
            srv_w_at(wave, k, 0)[o] = w[0];
            srv_w_at(wave, k, 1)[o] = w[1];
        }
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

#if SP_MERGE_QUERIES
// mis_material_part (estimate_direct_mis after its shadow ray, Integrator.cpp:505-535) with the MIS
// ray's occlusion test left to the merged pass: true when its BVH walk was posted (origin,
// direction, t_min in the owner's MQ_O / MQ_D3 / MQ_T3 slots).  e_occ is the estimate if that ray
// is occluded, e_vis if not (the MIS term is a pure function of values known now, computed with
// the same operations in the same order); otherwise the estimate is final in e_occ.  Counts and
// draws are mis_material_part's.
__device__ __forceinline__ bool mis_material_part_mq(Ctx& c, const Light& l, const LSample& ls, f3 p, f3 n, f3 wo, int mid,
                                                     uint32_t* m, rgb& e_occ, rgb& e_vis)
{
    const int lane = threadIdx.x & 63;
    rgb       Lr   = mkc(0, 0, 0);
    const f3  wi   = ls.ray.d;
    const rgb be   = material_eval(c.sc, mid, wo, wi, n, c.rng, c.q);
    if (!cblack(be)) {
        const float bp = material_pdf(c.sc, mid, wo, wi, n, c.rng, c.q);
        if (bp > 0.0f) {
            const float w = balance(ls.pdf, ls.pdf + bp);
            Lr            = cadd(Lr, cscale(cmul(be, ls.L), abs_f(dot(wi, n)) * w / ls.pdf));
        }
    }
    e_occ            = Lr;
    const MSample ms = material_sample(c.sc, mid, wo, n, c.rng, c.q);
    if (ms.pdf == 0.0f || cblack(ms.color)) return false;
    const float lp = light_pdf(c.sc, l, p, ms.dir);
    if (lp == 0.0f) return false;
    const float w = balance(ms.pdf, ms.pdf + lp);
    Ray         mr;
    mr.o             = p;
    mr.d             = ms.dir;
    const float mmin = ray_offset(n, ms.dir);
    ++c.rays;
    LightHit lh;
    SP_WPROF(3, lh = scene_intersect_lights(c.sc, mr, mmin, k_infinite, c.st));
    if (!lh.hit) return false;
    ++c.shadow; // occluded(): Scene::intersect_p = geometry (unbounded shapes, BVH) || lights
    ++c.rays;
    if (unbounded_any(c.sc, mr, mmin, k_infinite)) return false; // occluded
    e_vis = cadd(Lr, cdivs(cscale(cscale(cmul(ms.color, light_hit_L(c.sc, lh, mr.d, c.q)), abs_f(dot(ms.dir, n))), w), ms.pdf));
    if (c.sc.n_nodes == 0) {
        if (!lights_any(c.sc, mr, mmin, k_infinite, c.st)) e_occ = e_vis;
        return false;
    }
    mq_put3(m, MQ_O, lane, p);
    mq_put3(m, MQ_D3, lane, ms.dir);
    m[MQ_T3 + lane]  = __float_as_uint(mmin);
    m[MQ_ANY + lane] = 0u;
    return true;
}
// mis_light_part (Integrator.cpp:496-502: Light::sample, then the shadow ray's intersect_p) with the
// shadow ray's BVH walk shared by the wave: every lane of integrate() calls it (want: this lane has
// a hit to estimate light l at).  Same draws, counts and result as mis_light_part.
__device__ __forceinline__ bool mis_light_part_mq(Ctx& c, const Light& l, f3 p, f3 n, LSample& ls, bool want, uint32_t* m)
{
    const int lane = threadIdx.x & 63;
    bool      go = false, post = false;
    if (want) {
        ls = light_sample(c.sc, l, p, n, next2D(c.rng), c.q);
        if (!(ls.pdf == 0.0f || cblack(ls.L))) {
            ++c.shadow; // occluded(): geometry (unbounded shapes, BVH) || lights
            ++c.rays;
            if (!unbounded_any(c.sc, ls.ray, ls.tmin, ls.tmax)) {
                if (c.sc.n_nodes == 0) {
                    go = !lights_any(c.sc, ls.ray, ls.tmin, ls.tmax, c.st);
                } else {
                    mq_put3(m, MQ_O, lane, ls.ray.o);
                    mq_put3(m, MQ_D3, lane, ls.ray.d);
                    m[MQ_T3 + lane]   = __float_as_uint(ls.tmin);
                    m[MQ_BEST + lane] = __float_as_uint(ls.tmax);
                    m[MQ_ANY + lane]  = 0u;
                    post              = true;
                }
            }
        }
    }
    const uint64_t mp = __ballot(post);
    if (mp != 0ull) {
        if (post) reinterpret_cast<uint8_t*>(m + MQ_Q)[__popcll(mp & ((1ull << lane) - 1ull))] = (uint8_t)(lane | 0x80);
        mq_sync();
        SP_WPROF(5, mq_run<MqLayout>(c.sc, c.st, m, __popcll(mp), true));
        if (post) go = !(m[MQ_ANY + lane] != 0u || lights_any(c.sc, ls.ray, ls.tmin, ls.tmax, c.st));
        mq_sync(); // the slots are serve_rho's next
    }
    return go;
}
// after mq_run: the MIS ray's Scene::intersect_p = the BVH walk's result || the lights
__device__ __forceinline__ bool mis_ray_occluded(Ctx& c, const uint32_t* m)
{
    const int lane = threadIdx.x & 63;
    if (m[MQ_ANY + lane] != 0u) return true;
    Ray mr;
    mr.o = mq_f3(m, MQ_O, lane);
    mr.d = mq_f3(m, MQ_D3, lane);
    return lights_any(c.sc, mr, mq_f(m, MQ_T3 + lane), k_infinite, c.st);
}
#endif

// IntegratorIterativeRRNEE (Integrators/Integrator.cpp:550) with wave-served estimates: the same
// per-lane operations as the form below, but a lane whose path has ended stays in the loop (no
// break) so that every lane of the wave is there to serve estimates.
__device__ __forceinline__ rgb integrate_rrnee(Ctx& c, Ray ray)
{
    rgb   throughput = mkc(1, 1, 1);
    rgb   L          = mkc(0, 0, 0);
    float tmin = k_ray_epsilon, tmax = k_infinite;
    constexpr float rr_cut = 0.1f;
    bool  alive = true;
    Query qr;
#if SP_MERGE_QUERIES
    // merged query pass (mq_run) on scenes whose closest hits walk the 8-wide BVH with the LDS
    // stack (SAH uploads); the reference-order BVH and stackless walks keep the per-lane queries
    const bool mq     = c.sc.merge_queries != 0 && c.sc.wide_closest != 0 && !c.sc.stackless;
    uint32_t*  m      = srv_lds[threadIdx.x >> 6];
    bool       traced = false; // this bounce's closest hit came from the previous merged pass
#endif
    for (int depth = 0; depth < c.sc.max_depth; ++depth) {
        if (!__any(alive)) break;
        // lock-step efficiency: wave bounce iterations (lines slot) and the lanes alive in them
        SP_TD(td_add(TD_BOUNCE, 1, (uint64_t)__popcll(__ballot(alive))));
        MSample s;
        f3      wo  = mk(0, 0, 0), n = mk(0, 0, 0);
        bool    hit = false, pend = false;
        Rng     snap = c.rng;
#if SP_MERGE_QUERIES
        bool tail = false, post1 = false;
        rgb  L_vis = mkc(0, 0, 0); // tail: L if the last light's MIS ray is unoccluded (L itself: if occluded)
#endif
        if (alive) {
            rng_prepare(c.rng);
#if SP_MERGE_QUERIES
            if (!traced)
#endif
            qr = trace(c, ray, tmin, tmax);
            if (qr.geom) {
                wo = neg(ray.d);
                n  = qr.is.n;
#if SP_SERVE_SAMPLE
                // The bounce's Material::sample estimate joins the first light's served estimates:
                // the sample's words are skipped now and the call runs from here with the served
                // weights after the first light's shadow ray.
                // The whole bounce (at most 1 + 32 + 3 + 2 + 97 words up to that light's sample
                // estimate) is reserved first, so none of these words is twisted over meanwhile.
                const bool defer = c.sc.n_lights > 0 && material_has_rho(c.sc, qr.is.material);
                if (defer) {
                    rng_reserve(c.rng, 140);
                    snap = c.rng;
                    // material_sample_local's draws without its arithmetic: a clearcoat's Fresnel
                    // pick first (a specular pick is drawn again below, from snap, and computed now)
                    const Material& mm   = c.sc.materials[qr.is.material];
                    const f3        wl   = to_onb(onb_from_v(n, c.q), wo);
                    bool            spec = false;
                    if (mm.kind == SP_MAT_CLEARCOAT) spec = next1D(c.rng) < fresnel_dielectric(wl.y, 1.0f, mm.coat_ior);
                    if (spec) {
                        c.rng = snap;
                    } else {
                        // the estimate starts here; after it the sample draws three words whichever
                        // lobe it picks (the glossy lobe draws none only when wo.y == 0, and then its
                        // weight is 0)
                        pend           = true;
                        c.rng.srv_dc   = (wl.y == 0.0f) ? 0u : 32u;
                        c.rng.srv_posA = c.rng.draws;
                        c.rng.srv_pwA  = ((uint32_t)c.rng.cur << 16) | (uint32_t)c.rng.idx;
                        rng_skip_reserved(c.rng, (int)c.rng.srv_dc + 3);
                    }
                }
                if (!pend)
#endif
                s = material_sample(c.sc, qr.is.material, wo, n, c.rng, c.q);
                if (pend) hit = true; // whether the sample is usable is known once it is finished
                else if (s.pdf == 0.0f || cblack(s.color)) alive = false;
                else hit = true;
            } else {
                if (qr.lh.hit) L = cadd(L, cmul(throughput, light_hit_L(c.sc, qr.lh, ray.d, c.q)));
                alive = false;
            }
        }
        for (int li = 0; li < c.sc.n_lights; ++li) {
            LSample        ls;
            bool           go = false, want = false;
            const uint32_t rays0 = c.rays, shadow0 = c.shadow;
#if SP_MERGE_QUERIES && SP_MQ_SHADOW
            if (mq) {
                go   = mis_light_part_mq(c, c.sc.lights[li], qr.is.p, n, ls, hit, m);
                want = go && material_has_rho(c.sc, qr.is.material);
            } else
#endif
            if (hit) {
                go   = mis_light_part(c, c.sc.lights[li], qr.is.p, n, ls);
                want = go && material_has_rho(c.sc, qr.is.material);
            }
            serve_rho(c, want, li == 0 && pend, (want || pend) ? qr.is.material : 0, n, wo);
#if SP_SERVE_SAMPLE
            if (li == 0 && pend) {
                // the deferred Material::sample, from the bounce's stream position, now with its weights
                Rng ra      = snap;
                ra.srv_on   = 1;
                ra.srv_A    = true;
                ra.srv_B    = false;
                ra.srv_posA = c.rng.srv_posA;
                ra.srv_dc   = c.rng.srv_dc;
                s           = material_sample(c.sc, qr.is.material, wo, n, ra, c.q);
                c.rng.srv_A = false;
                if (s.pdf == 0.0f || cblack(s.color)) {
                    // not usable: the path ends right after the sample (Integrator.cpp:566), so the
                    // light's sample and shadow ray never happened -- stream and counters go back
                    ra.srv_on = 0;
                    ra.srv_A  = false;
                    c.rng     = ra;
                    c.rays    = rays0;
                    c.shadow  = shadow0;
                    hit = go = alive = false;
                }
            }
#endif
            if (hit) {
                rgb e = mkc(0, 0, 0);
#if SP_MERGE_QUERIES
                rgb e_vis = mkc(0, 0, 0);
                if (go && mq && li == c.sc.n_lights - 1) // the last light's MIS ray joins the merged pass
                    tail = mis_material_part_mq(c, c.sc.lights[li], ls, qr.is.p, n, wo, qr.is.material, m, e, e_vis);
                else
#endif
                if (go) e = mis_material_part(c, c.sc.lights[li], ls, qr.is.p, n, wo, qr.is.material);
                c.rng.srv_on   = 0;
                c.rng.srv_B    = false;
#if SP_MERGE_QUERIES
                if (tail) L_vis = cadd(L, cmul(throughput, e_vis));
#endif
                L = cadd(L, cmul(throughput, e));
            }
        }
        if (hit) {
            const f3    next_o = ray_at(ray, qr.is.t);
            const f3    wi     = s.dir;
            const float cosine = abs_f(dot(wi, n));
            throughput         = cmul(throughput, cdivs(cscale(s.color, cosine), s.pdf));
            if (depth >= c.sc.rr_depth) {
                const float lum = luminance(throughput);
                if (lum < rr_cut) {
                    const float qv = std_max(0.05f, lum / rr_cut);
                    if (next1D(c.rng) < qv) throughput = cdivs(throughput, qv);
                    else alive = false;
                }
            }
            ray.o = next_o;
            ray.d = wi;
            tmin  = ray_offset(cosine);
            tmax  = k_infinite;
#if SP_MERGE_QUERIES
            if (mq && alive && depth + 1 < c.sc.max_depth) {
                // the next bounce's trace(): intersect_lights and the unbounded shapes now, the BVH
                // walk in the merged pass (next_o is qr.is.p: ray_at of the same ray and t)
                ++c.rays;
                qr.lh          = scene_intersect_lights(c.sc, ray, tmin, tmax, c.st);
                const float tm = qr.lh.hit ? qr.lh.t : tmax;
                const Hit   h0 = scene_intersect_unbounded(c.sc, ray, tmin, tm);
                const int   ln = threadIdx.x & 63;
                mq_put3(m, MQ_O, ln, ray.o);
                mq_put3(m, MQ_D1, ln, ray.d);
                m[MQ_T1 + ln]      = __float_as_uint(tmin);
                *mq_best<MqLayout>(m, ln)    = ((unsigned long long)__float_as_uint(h0.t) << 32) | 0xffffffffull;
                post1              = true;
            }
#endif
        }
#if SP_MERGE_QUERIES
        traced = false;
        if (mq) {
            const uint64_t m1 = __ballot(post1), m3 = __ballot(tail);
            if ((m1 | m3) != 0ull) {
                const int      ln = threadIdx.x & 63;
                const uint64_t lt = (1ull << ln) - 1ull;
                const int      n1 = __popcll(m1);
                uint8_t*       qs = reinterpret_cast<uint8_t*>(m + MQ_Q);
                if (post1) qs[__popcll(m1 & lt)] = (uint8_t)ln;
                if (tail) qs[n1 + __popcll(m3 & lt)] = (uint8_t)(ln | 0x80);
                mq_sync();
                SP_WPROF(5, mq_run<MqLayout>(c.sc, c.st, m, n1 + __popcll(m3)));
                if (tail && !mis_ray_occluded(c, m)) L = L_vis;
                if (post1) {
                    // the walk's answer: (t, wide slot) of the closest BVH primitive, or the
                    // unbounded shapes' hit; the primitive's test is repeated for its code, beta, gamma
                    const unsigned long long key = *mq_best<MqLayout>(m, ln);
                    const uint32_t slot = (uint32_t)key;
                    Hit h;
                    if (slot == 0xffffffffu) {
                        h = scene_intersect_unbounded(c.sc, ray, tmin, qr.lh.hit ? qr.lh.t : tmax);
                    } else {
                        h.t = k_infinite; h.code = 0xffffffffu; h.slot = 0xffffffffu;
                        prim_closest_w(c.sc, slot, ray, tmin, h);
                    }
                    qr.geom = (h.code != 0xffffffffu);
                    if (qr.geom) qr.is = finish_hit(c.sc, h, ray, c.q);
                    traced = true;
                }
                mq_sync(); // the slots are the next serve_rho round's
            }
        }
#endif
    }
    return L;
}

#else
// IntegratorIterativeRRNEE (Integrators/Integrator.cpp:550)
__device__ __forceinline__ rgb integrate_rrnee(Ctx& c, Ray ray)
{
    rgb   throughput = mkc(1, 1, 1);
    rgb   L          = mkc(0, 0, 0);
    float tmin = k_ray_epsilon, tmax = k_infinite;
    constexpr float rr_cut = 0.1f;
    for (int depth = 0; depth < c.sc.max_depth; ++depth) {
        rng_prepare(c.rng);
        const Query qr = trace(c, ray, tmin, tmax);
        if (qr.geom) {
            const f3      wo = neg(ray.d);
            const f3      n  = qr.is.n;
            const MSample s  = material_sample(c.sc, qr.is.material, wo, n, c.rng, c.q);
            if (s.pdf == 0.0f || cblack(s.color)) break;
            for (int li = 0; li < c.sc.n_lights; ++li)
                L = cadd(L, cmul(throughput, estimate_direct_mis(c, c.sc.lights[li], qr.is.p, n, wo, qr.is.material)));
            const f3    next_o = ray_at(ray, qr.is.t);
            const f3    wi     = s.dir;
            const float cosine = abs_f(dot(wi, n));
            throughput         = cmul(throughput, cdivs(cscale(s.color, cosine), s.pdf));
            if (depth >= c.sc.rr_depth) {
                const float lum = luminance(throughput);
                if (lum < rr_cut) {
                    const float qv = std_max(0.05f, lum / rr_cut);
                    if (next1D(c.rng) < qv) throughput = cdivs(throughput, qv);
                    else break;
                }
            }
            ray.o = next_o;
            ray.d = wi;
            tmin  = ray_offset(cosine);
            tmax  = k_infinite;
        } else if (qr.lh.hit) {
            L = cadd(L, cmul(throughput, light_hit_L(c.sc, qr.lh, ray.d, c.q)));
            break;
        } else {
            break;
        }
    }
    return L;
}
#endif

// ============================================================================ the kernel
// MandelbrotIntegrator::integrate_impl + mandel (Integrators/Integrator.cpp:59-105) with
// to_rgb (math/HSV.h:133, the active #else branch).  No scene queries, no sampler draws.
__device__ __forceinline__ rgb integrate_mandelbrot(float px, float py, int W, int H)
{
    const float x0 = -2.0f, x1 = 1.0f, y0 = -1.0f, y1 = 1.0f;
    const float dx = (x1 - x0) / (float)W;
    const float dy = (y1 - y0) / (float)H;
    const float cre = x0 + px * dx, cim = y0 + py * dy;
    float       zr = cre, zi = cim;
    int         it = 0;
    for (; it < 4096; ++it) { // s_max_iterations (Integrator.h:69)
        if (zr * zr + zi * zi > 4.0f) break;
        const float nr = zr * zr - zi * zi;
        const float ni = 2.0f * zr * zi;
        zr             = cre + nr;
        zi             = cim + ni;
    }
    const float value = (float)it / (float)4096;
    const float hue   = fmodf(lm_powf(value * 360.0f, 1.5f), 360.0f) / 360.0f; // fmod is exact
    const float C     = value * 1.0f;
    const int   hp    = (int)floorf(hue * 6.0f);
    // std::fmod(int, float) promotes to double: X = C * (1 - |hp mod 2 - 1|) = hp odd ? C : 0
    const float X = (hp & 1) ? C : 0.0f * C;
    switch (hp % 6) {
    case 0: return mkc(C, X, 0);
    case 1: return mkc(X, C, 0);
    case 2: return mkc(0, C, X);
    case 3: return mkc(0, X, C);
    case 4: return mkc(X, 0, C);
    case 5: return mkc(C, 0, X);
    }
    return mkc(0, 0, 0);
}

__device__ __forceinline__ uint32_t morton_decode_1(uint32_t a)
{
    a = a & 0x55555555u;
    a = (a | (a >> 1)) & 0x33333333u;
    a = (a | (a >> 2)) & 0x0F0F0F0Fu;
    a = (a | (a >> 4)) & 0x00FF00FFu;
    a = (a | (a >> 8)) & 0x0000FFFFu;
    return a;
}

} // inline namespace SPD_LAYOUT_NS
} // namespace spd
