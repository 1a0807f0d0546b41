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

// variant = requested waves per SIMD for __launch_bounds__ (1..4, DirectLighting only); 0 = default
KernelFn select_kernel(int integ, int variant)
{
    switch (integ) {
    case SP_INTEGRATOR_BRUTE_FORCE:
    case SP_INTEGRATOR_WHITTED: return mega_recursive(integ);
    case SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE:
    case SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE_RR: return mega_iterative(integ, regen_env());
    case SP_INTEGRATOR_ITERATIVE_RRNEE: return mega_rrnee(regen_env());
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

int render_blocks_per_cu(int integ, int variant, size_t lds_bytes)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, select_kernel(integ, variant), 64 * WAVES_PER_BLOCK, lds_bytes) !=
        hipSuccess)
        return 1;
    return n > 0 ? n : 1;
}

} // namespace spd
