// sp_mega.hip -- launch helpers of the megakernel (sp_mega.hpp); kernels live in sp_mega_*.hip.
#include "sp_mega.hpp"

namespace spd {

// variant = requested waves per SIMD for __launch_bounds__ (DirectLighting 1..4, IterativeRRNEE 2..4)
KernelFn select_kernel(int integ, int variant)
{
    switch (integ) {
    case SP_INTEGRATOR_BRUTE_FORCE:
    case SP_INTEGRATOR_WHITTED: return mega_recursive(integ);
    case SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE:
    case SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE_RR: return mega_iterative(integ);
    case SP_INTEGRATOR_ITERATIVE_RRNEE: return mega_rrnee(variant);
    case SP_INTEGRATOR_MANDELBROT: return mega_mandelbrot();
    default: return mega_direct(variant);
    }
}

hipError_t launch_render(const Scene& sc, const RenderArgs& args, int integ, int variant, int blocks, size_t lds_bytes,
                         hipStream_t stream)
{
    hipLaunchKernelGGL(select_kernel(integ, variant), dim3(blocks), dim3(64 * WAVES_PER_BLOCK), lds_bytes, stream, sc, args);
    return hipGetLastError();
}

// the probe kernel of an integrator's megakernel (tile order below); nullptr: none built
static KernelFn select_probe(int integ, int variant)
{
    if (integ == SP_INTEGRATOR_DIRECT_LIGHTING) return probe_direct(variant);
    if (integ == SP_INTEGRATOR_ITERATIVE_RRNEE) return probe_rrnee(variant);
    return nullptr;
}
bool has_probe(int integ) { return select_probe(integ, 0) != nullptr; }
hipError_t launch_probe(const Scene& sc, const RenderArgs& args, int integ, int variant, int blocks, size_t lds_bytes,
                        hipStream_t stream)
{
    const KernelFn k = select_probe(integ, variant);
    if (!k) return hipErrorInvalidDeviceFunction;
    hipLaunchKernelGGL(k, dim3(blocks), dim3(64 * WAVES_PER_BLOCK), lds_bytes, stream, sc, args);
    return hipGetLastError();
}

// Tile order for the persistent megakernel.  Each wave renders its tiles one after another, and a
// tile's cost spans two orders of magnitude (bunny 1080p @ 256 spp: 1 ms of sky to 234 ms of
// glossy floor under a bunny); in queue order the most expensive tiles can be taken late, and the
// frame ends with a tail in which a few waves finish them alone (profiles/r03/tile_timeline_*:
// the last 15 % of the span ran below full occupancy, 9 % of the frame).  A probe pass renders
// one sample of every tile (sp_probe_kernel with spp = 1: the render's code writing tile times
// instead of radiance; the render re-seeds every pixel's stream) and times each tile; this kernel
// then orders the queue by cost class: the tiles whose cost estimate exceeds `factor` x the mean
// first, then those above factor r, factor r^2, ... x the mean (SP_TILE_CLASSES classes, ratio r =
// SP_TILE_RATIO, the last holding the rest).  Each class keeps queue order (a stable counting sort),
// so consecutive tiles of one class stay spatially coherent -- which a full longest-first sort loses
//  -- and the cheapest tiles are taken last, where they fill the frame's tail.
// Round 4 (§10l): 6 classes an octave apart.  Round 5 (§11l): replaying the measured bunny timeline
// as list scheduling showed that the octave-wide classes themselves left the tail (a 30 ms tile of
// the 15-31 ms class taken at 230 ms; tools/tile_sched_sim.py): 24 classes a quarter octave apart
// measured bunny +0.3 %, lucy +1.6 %, elf's 8-way shard +1.6-3.5 % (elf: single-frame runs, --steps 1
// --warmup 0; re-measured with warm-up and 2 steps in DESIGN.md §12).
// Only which wave takes which tile, and when, changes: every pixel's result is the same.
#ifndef SP_TILE_CLASSES
#define SP_TILE_CLASSES 24
#endif
constexpr int TILE_CLASSES = SP_TILE_CLASSES;
#ifndef SP_TILE_RATIO
#define SP_TILE_RATIO 0.84089642f // 2^(-1/4)
#endif
__device__ __forceinline__ int tile_class(float t, float thr)
{
    int k = 0;
#pragma unroll
    for (int j = 0; j + 1 < TILE_CLASSES; ++j, thr *= SP_TILE_RATIO) k += t > thr ? 0 : 1;
    return k; // 0: slower than thr; class j + 1: not slower than thr r^j
}
#ifndef SP_TILE_SMOOTH
#define SP_TILE_SMOOTH 1
#endif
// A tile's cost estimate: its one-sample probe time blended with its image neighbours', against
// the probe's noise -- the larger of the row blend (left, right) and the column blend (above,
// below), so a tile next to an expensive region is not taken late.  tx: the queue offset of the
// tile below (> 0), -1 when only the +-1 queue entries are used, < -1 the column blend alone with
// offset -tx - 1, 0 none (a caller's list in arbitrary order: the probe time alone); the +-1 entries
// are the left / right tiles of a whole frame and k tiles apart in a stride-k list
// (sp_capi.hip order_neighbours).
// Measured against the row blend alone (round 4's form) and the probe time alone: lucy +0.9-1.5 %,
// elf's 8-way shard +1.3 %, bunny level (profiles/r05/tile_order/).  SP_TILE_SMOOTH 0: probe time alone.
__device__ __forceinline__ float tile_est(const float* t, int64_t i, int64_t n, int tx)
{
    if (!SP_TILE_SMOOTH || tx == 0) return t[i];
    if (tx < -1) {
        const int64_t o = -(int64_t)tx - 1;
        const float   u = t[i >= o ? i - o : i], d = t[i + o < n ? i + o : i];
        return 0.25f * (u + d) + 0.5f * t[i];
    }
    const float l = t[i > 0 ? i - 1 : i], r = t[i + 1 < n ? i + 1 : i];
    const float row = 0.25f * (l + r) + 0.5f * t[i];
    if (tx < 0) return row;
    const float u = t[i >= tx ? i - tx : i], d = t[i + tx < n ? i + tx : i];
    return fmaxf(row, 0.25f * (u + d) + 0.5f * t[i]);
}
__global__ void __launch_bounds__(1024) tile_order_kernel(float* tile_time, int64_t n, float factor, int tx, int step,
                                                          int32_t* order)
{
    __shared__ float s_sum[16];
    __shared__ int   s_cnt[TILE_CLASSES][16];
    __shared__ int   s_base[TILE_CLASSES];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    // a probe of every step-th slot: the others from their probed queue neighbours (linear)
    if (step > 1) {
        for (int64_t i = tid; i < n; i += 1024) {
            const int64_t r = i % step;
            if (r == 0) continue;
            const int64_t lo = i - r, hi = lo + step;
            tile_time[i] = hi < n ? tile_time[lo] + (tile_time[hi] - tile_time[lo]) * ((float)r / (float)step) : tile_time[lo];
        }
        __syncthreads();
    }
    float     sum = 0.0f;
    for (int64_t i = tid; i < n; i += 1024) sum += tile_time[i];
    for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off, 64);
    if (lane == 0) s_sum[wave] = sum;
    __syncthreads();
    float total = 0.0f;
    for (int w = 0; w < 16; ++w) total += s_sum[w];
    const float thr = factor * total / (float)n;
    // class sizes (one pass, LDS histogram) -> each class's first position (classes in order 0, 1, ...)
    __shared__ int s_hist[TILE_CLASSES];
    for (int k = tid; k < TILE_CLASSES; k += 1024) s_hist[k] = 0;
    __syncthreads();
    for (int64_t i = tid; i < n; i += 1024) atomicAdd(&s_hist[tile_class(tile_est(tile_time, i, n, tx), thr)], 1);
    __syncthreads();
    if (tid == 0) {
        int b = 0;
        for (int k = 0; k < TILE_CLASSES; ++k) {
            s_base[k] = b;
            b += s_hist[k];
        }
    }
    __syncthreads();
    for (int64_t c0 = 0; c0 < n; c0 += 1024) {
        const int64_t i   = c0 + tid;
        const bool    v   = i < n;
        const int     cls = v ? tile_class(tile_est(tile_time, i, n, tx), thr) : -1;
        uint32_t      pos = 0;
        for (int k = 0; k < TILE_CLASSES; ++k) {
            const uint64_t  m = __ballot(cls == k);
            const uint32_t  p = __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
            if (cls == k) pos = p;
            if (lane == 0) s_cnt[k][wave] = __popcll(m);
        }
        __syncthreads();
        if (v) {
            int o = s_base[cls];
            for (int w = 0; w < wave; ++w) o += s_cnt[cls][w];
            order[o + (int)pos] = (int32_t)i;
        }
        __syncthreads();
        if (tid == 0)
            for (int k = 0; k < TILE_CLASSES; ++k)
                for (int w = 0; w < 16; ++w) s_base[k] += s_cnt[k][w];
        __syncthreads();
    }
}

hipError_t launch_tile_order(float* tile_time, int64_t n_tiles, float factor, int tiles_x, int step, int32_t* order,
                             hipStream_t stream)
{
    hipLaunchKernelGGL(tile_order_kernel, dim3(1), dim3(1024), 0, stream, tile_time, n_tiles, factor, tiles_x, step, order);
    return hipGetLastError();
}

// Static LDS of a render kernel (libm tables, the rho sink, IterativeRRNEE's served-estimate
// rows): the 160 KB guard and the LDS occupancy cap count it beside the dynamic part.
size_t render_static_lds(int integ, int variant)
{
    hipFuncAttributes fa{};
    if (hipFuncGetAttributes(&fa, reinterpret_cast<const void*>(select_kernel(integ, variant))) != hipSuccess) return 0;
    return fa.sharedSizeBytes;
}

// variant 0: the sample chunks' fused form (sp_fused_kernel), 3 / 4: the tail kernel at 3 / 4 waves,
// -4: the tail kernel with an image light's replay (4 waves)
static KernelFn tail_kernel(int variant)
{
    return variant == 0 ? fused_chunks() : tail_direct(variant < 0 ? -variant : variant, variant < 0);
}
hipError_t launch_tail(const Scene& sc, const RenderArgs& args, int variant, int blocks, size_t lds_bytes, hipStream_t stream)
{
    hipLaunchKernelGGL(tail_kernel(variant), dim3(blocks), dim3(64 * WAVES_PER_BLOCK), lds_bytes, stream, sc, args);
    return hipGetLastError();
}
int tail_blocks_per_cu(int variant, size_t lds_bytes)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, tail_kernel(variant), 64 * WAVES_PER_BLOCK, lds_bytes) != hipSuccess) return 1;
    return n > 0 ? n : 1;
}

int render_blocks_per_cu(int integ, int variant, size_t lds_bytes)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, select_kernel(integ, variant), 64 * WAVES_PER_BLOCK, lds_bytes) !=
        hipSuccess)
        return 1;
    return n > 0 ? n : 1;
}

} // namespace spd
