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

int render_blocks_per_cu(int integ, int variant, size_t lds_bytes)
{
    int n = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, select_kernel(integ, variant), 64 * WAVES_PER_BLOCK, lds_bytes) !=
        hipSuccess)
        return 1;
    return n > 0 ? n : 1;
}

} // namespace spd
