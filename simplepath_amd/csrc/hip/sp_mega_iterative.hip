// sp_mega_iterative.hip -- BruteForceIntegratorIterative(RR) megakernels.
#include "sp_mega.hpp"

#include <cstdlib>

namespace spd {
// regen = per-lane sample regeneration (sp_render_regen, default); 0 = lock-step samples
KernelFn mega_iterative(int integ, bool regen)
{
    if (integ == SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE_RR)
        return regen ? sp_render_regen<SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE_RR, 2> : sp_render_kernel<SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE_RR, 2>;
    return regen ? sp_render_regen<SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE, 2> : sp_render_kernel<SP_INTEGRATOR_BRUTE_FORCE_ITERATIVE, 2>;
}
} // namespace spd
