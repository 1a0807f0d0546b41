// sp_mega_rrnee.hip -- IterativeIntegratorRRNEE megakernels: lock-step with merged selection-weight
// estimates, and lock-step plain (default).
#include "sp_mega.hpp"

namespace spd {
KernelFn mega_rrnee(bool merged, int w)
{
    // Built without SLP vectorisation the per-call-site kernel fits 243 VGPRs with no scratch and
    // is the faster form (elf 1024^2 x 16 spp: 479 vs 452 Mrays/s merged, profiles/r02/s5); the
    // merged form (SP_RRNEE_MERGED=1) won while both spilled (440 vs 395).
    // w = waves per SIMD (sp_render_tiles: 3 unless SP_KERNEL_VARIANT or the LDS says otherwise);
    // elf 1024^2 x 16 spp: 476 / 553 / 519 Mrays/s at 2 / 3 / 4 waves (profiles/r02/s5)
    if (merged) return w == 2 ? sp_render_kernel<INTEG_RRNEE_MERGED, 2> : sp_render_kernel<INTEG_RRNEE_MERGED, 3>;
    if (w == 2) return sp_render_kernel<SP_INTEGRATOR_ITERATIVE_RRNEE, 2>;
    if (w == 4) return sp_render_kernel<SP_INTEGRATOR_ITERATIVE_RRNEE, 4>;
    return sp_render_kernel<SP_INTEGRATOR_ITERATIVE_RRNEE, 3>;
}
} // namespace spd
