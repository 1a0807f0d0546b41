// sp_mega_direct.hip -- DirectLighting megakernel instantiations (__launch_bounds__ variants).
#include "sp_mega.hpp"

namespace spd {
KernelFn mega_direct(int variant)
{
    switch (variant) {
    case 1: return sp_render_kernel<SP_INTEGRATOR_DIRECT_LIGHTING, 1>;
    case 3: return sp_render_kernel<SP_INTEGRATOR_DIRECT_LIGHTING, 3>;
    case 4: return sp_render_kernel<SP_INTEGRATOR_DIRECT_LIGHTING, 4>;
    default: return sp_render_kernel<SP_INTEGRATOR_DIRECT_LIGHTING, 2>;
    }
}
KernelFn mega_mandelbrot() { return sp_render_kernel<SP_INTEGRATOR_MANDELBROT, 2>; }
} // namespace spd
