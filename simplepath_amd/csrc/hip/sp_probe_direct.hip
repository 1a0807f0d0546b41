// sp_probe_direct.hip -- tile-order probe kernels of the DirectLighting megakernel (sp_mega.hpp
// sp_probe_kernel), built with sp_mega_direct.hip's settings so a probe tile costs what the
// render's tile does; a translation unit of their own so they compile beside the render kernels.
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
KernelFn probe_direct(int variant)
{
    switch (variant) {
    case 1: return sp_probe_kernel<SP_INTEGRATOR_DIRECT_LIGHTING, 1>;
    case 2: return sp_probe_kernel<SP_INTEGRATOR_DIRECT_LIGHTING, 2>;
    case 3: return sp_probe_kernel<SP_INTEGRATOR_DIRECT_LIGHTING, 3>;
    default: return sp_probe_kernel<SP_INTEGRATOR_DIRECT_LIGHTING, 4>;
    }
}
} // namespace spd
