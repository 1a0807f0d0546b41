// sp_mega_rrnee.hip -- IterativeIntegratorRRNEE megakernel.
#include "sp_mega.hpp"

namespace spd {
KernelFn mega_rrnee() { return sp_render_kernel<SP_INTEGRATOR_ITERATIVE_RRNEE, 2>; }
} // namespace spd
