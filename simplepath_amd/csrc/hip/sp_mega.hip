// sp_mega.hip -- launch helpers of the megakernel (sp_mega.hpp); kernels live in sp_mega_*.hip.
#include "sp_mega.hpp"

#include <cstdlib>

namespace spd {

// SP_REGEN=1 selects per-lane sample regeneration (sp_render_regen) for the iterative
// integrators.  Opt-in: on elf.sp (1024x1024, 16 spp, IterativeRRNEE) it measured 254 Mrays/s
// against 324 for the lock-step loop -- mixing camera and bounce rays in a wave costs more
// traversal coherence than the lock step wastes on paths of ~1.2 bounces.
static bool regen_env()
{
    const char* v = std::getenv("SP_REGEN");
    return v ? std::atoi(v) != 0 : false;
}

// SP_RRNEE_MERGED=1: the lock-step IterativeRRNEE megakernel with the selection-weight estimates
// merged across call sites (sp_path.hpp integrate_rrnee_merged; identical images).  It won while
// both forms spilled (440 vs 395 Mrays/s on elf 1024^2 x 16 spp); built without SLP
// vectorisation the per-call-site form needs no scratch and is faster (479 vs 452).
static bool rrnee_merged_env()
{
    const char* v = std::getenv("SP_RRNEE_MERGED");
    return v ? std::atoi(v) != 0 : false;
}

// variant = requested waves per SIMD for __launch_bounds__ (DirectLighting 1..4, IterativeRRNEE 2..4)
KernelFn select_kernel(int integ, int variant)
{
    switch (integ) {
    case SP_INTEGRATOR_BRUTE_FORCE:
    case SP_INTEGRATOR_WHITTED: return mega_recursive(integ);
    case SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE:
    case SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE_RR: return mega_iterative(integ, regen_env());
    case SP_INTEGRATOR_ITERATIVE_RRNEE: return mega_rrnee(regen_env(), rrnee_merged_env(), variant);
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

// Tile cost probe: one centre ray per pixel; a tile's cost estimate is what its wave will pay per
// sample -- the most expensive material among its lanes (SIMD lanes wait for the slowest) plus a
// little per hit.  Weights: glossy base (16-sample rho estimate per light sample) 16, Lambertian
// or clearcoat-over-Lambertian 2, miss 0.  Used only to order the megakernel's tile queue
// (longest first), never to change what a tile computes.
__global__ void __launch_bounds__(256) tile_cost_kernel(Scene sc, const int32_t* tile_ids, int64_t n_tiles, int32_t tiles_x,
                                                        float* cost)
{
    extern __shared__ uint32_t lds[];
    const int64_t  slot = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6);
    const uint32_t lane = threadIdx.x & 63u;
    if (slot >= n_tiles) return;
    const Stack    st{ lds + (threadIdx.x >> 6) * sc.stack_words * 64, (int)lane, sc.stack_depth };
    const Rsq      q{ sc.rsqrt_entries, sc.rsqrt_bits, sc.rsqrt_zero, sc.rsqrt_denorm, sc.rsqrt_shift, sc.rsqrt_hi };
    const int32_t  tile = tile_ids ? tile_ids[slot] : (int32_t)slot;
    const uint32_t px   = (uint32_t)((tile % tiles_x) * 8) + morton_decode_1(lane);
    const uint32_t py   = (uint32_t)((tile / tiles_x) * 8) + morton_decode_1(lane >> 1);
    float          w    = 0.0f;
    if ((int)px < sc.width && (int)py < sc.height) {
        Ray ray;
        ray.o = sc.camera.p;
        ray.d = normalize(add(add(scale((float)px + 0.5f, sc.camera.vx), scale((float)py + 0.5f, sc.camera.vy)), sc.camera.vz), q);
        const Hit h = scene_intersect(sc, ray, k_ray_epsilon, k_infinite, st);
        if (h.code != 0xffffffffu) {
            const Isect is = finish_hit(sc, h, ray, q);
            Material    m  = sc.materials[is.material];
            if (m.kind == SP_MAT_CLEARCOAT) m = sc.materials[m.base];
            w = (m.kind == SP_MAT_GLOSSY) ? 16.0f : 2.0f;
        }
    }
    float mx = w, sum = w;
    for (int off = 32; off > 0; off >>= 1) {
        mx = max(mx, __shfl_xor(mx, off, 64));
        sum += __shfl_xor(sum, off, 64);
    }
    if (lane == 0) cost[slot] = mx + sum / 64.0f;
}

hipError_t launch_tile_cost(const Scene& sc, const int32_t* tile_ids, int64_t n_tiles, int32_t tiles_x, float* cost,
                            hipStream_t stream)
{
    const size_t lds = (size_t)4 * sc.stack_words * 64 * 4;
    hipLaunchKernelGGL(tile_cost_kernel, dim3((unsigned)((n_tiles + 3) / 4)), dim3(256), lds, stream, sc, tile_ids, n_tiles,
                       tiles_x, cost);
    return hipGetLastError();
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
