// sp_mega_direct.hip -- DirectLighting megakernel instantiations (__launch_bounds__ variants).
// No RNG draw-ahead window here, but the glossy estimate's words are touched in advance
// (sp_path.hpp SP_RHO_TOUCH): 2762 vs 2720 Mrays/s with the window of 2 (profiles/r02/s5).
#define SP_RNG_PF 0
#ifndef SP_RHO_TOUCH
#define SP_RHO_TOUCH 1
#endif
// two consecutive draws at an even stream position: one 16-byte load (sp_path.hpp rng_raw2)
#ifndef SP_RNG_PAIR
#define SP_RNG_PAIR 1
#endif
#include "sp_mega.hpp"

namespace spd {
KernelFn mega_direct(int variant)
{
    // default 4 waves per SIMD (128 VGPRs) once the device code was built without SLP
    // vectorisation: bunny 1080p @ 256 spp 2533 / 2706 Mrays/s at 3 / 4 waves, 2-way shard 1823 /
    // 2116 / 2138 at 2 / 3 / 4 (profiles/r02/s5)
    switch (variant) {
    case 1: return sp_render_kernel<SP_INTEGRATOR_DIRECT_LIGHTING, 1>;
    case 2: return sp_render_kernel<SP_INTEGRATOR_DIRECT_LIGHTING, 2>;
    case 3: return sp_render_kernel<SP_INTEGRATOR_DIRECT_LIGHTING, 3>;
    default: return sp_render_kernel<SP_INTEGRATOR_DIRECT_LIGHTING, 4>;
    }
}
KernelFn mega_mandelbrot() { return sp_render_kernel<SP_INTEGRATOR_MANDELBROT, 2>; }
} // namespace spd
