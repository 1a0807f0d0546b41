// sp_mega_rrnee.hip -- IterativeIntegratorRRNEE megakernels (lock-step and per-lane regeneration).
#include "sp_mega.hpp"

namespace spd {
KernelFn mega_rrnee(bool regen)
{
    return regen ? sp_render_regen<SP_INTEGRATOR_ITERATIVE_RRNEE, 2> : sp_render_kernel<SP_INTEGRATOR_ITERATIVE_RRNEE, 2>;
}
} // namespace spd
