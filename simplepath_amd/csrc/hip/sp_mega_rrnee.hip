// sp_mega_rrnee.hip -- IterativeIntegratorRRNEE megakernels: lock-step with merged selection-weight
// estimates (default), lock-step plain, and per-lane regeneration.
#include "sp_mega.hpp"

namespace spd {
KernelFn mega_rrnee(bool regen, bool merged)
{
    // merged: 2 waves/SIMD with 276 B/lane of scratch measured 440 Mrays/s on elf 1024^2 x 16 spp;
    // 1 wave/SIMD (spills to AGPRs, no scratch) 285
    if (merged && !regen) return sp_render_kernel<INTEG_RRNEE_MERGED, 2>;
    return regen ? sp_render_regen<SP_INTEGRATOR_ITERATIVE_RRNEE, 2> : sp_render_kernel<SP_INTEGRATOR_ITERATIVE_RRNEE, 2>;
}
} // namespace spd
