// sp_mega_recursive.hip -- BruteForceIntegrator and WhittedIntegrator megakernels.
#include "sp_mega.hpp"

namespace spd {
KernelFn mega_recursive(int integ)
{
    if (integ == SP_INTEGRATOR_WHITTED) return sp_render_kernel<SP_INTEGRATOR_WHITTED, 2>;
    return sp_render_kernel<SP_INTEGRATOR_BRUTE_FORCE, 2>;
}
} // namespace spd
