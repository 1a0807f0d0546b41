// sp_probe_rrnee.hip -- tile-order probe kernels of the IterativeRRNEE megakernel (sp_mega.hpp
// sp_probe_kernel, same settings as sp_mega_rrnee.hip).
// Multiple-importance estimates served across the wave (sp_path.hpp serve_rho).
#ifndef SP_SERVE_RHO
#define SP_SERVE_RHO 1
#endif
#include "sp_mega.hpp"

namespace spd {
KernelFn probe_rrnee(int w)
{
    if (w == 2) return sp_probe_kernel<SP_INTEGRATOR_ITERATIVE_RRNEE, 2>;
    if (w == 4) return sp_probe_kernel<SP_INTEGRATOR_ITERATIVE_RRNEE, 4>;
    return sp_probe_kernel<SP_INTEGRATOR_ITERATIVE_RRNEE, 3>;
}
} // namespace spd
