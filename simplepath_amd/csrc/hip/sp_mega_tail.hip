// sp_mega_tail.hip -- the DirectLighting megakernel with tail chunks (sp_mega.hpp tail_prep /
// tail_chunk, sp_device.hpp TailArgs), built with sp_mega_direct.hip's settings: no draw-ahead
// window, the glossy estimate's words touched in advance, paired draws.  4 waves per SIMD (the
// render's default) and 3 (the default where a deep BVH's LDS stacks cap the occupancy); other
// requested variants render without tail chunks.
#define SP_RNG_PF 0
#ifndef SP_RHO_TOUCH
#define SP_RHO_TOUCH 1
#endif
#ifndef SP_RNG_PAIR
#define SP_RNG_PAIR 1
#endif
#include "sp_mega.hpp"

namespace spd {
KernelFn tail_direct(int variant, bool replay)
{
    if (replay) return sp_tail_kernel<4, true>;
    return variant == 3 ? sp_tail_kernel<3, false> : sp_tail_kernel<4, false>;
}
KernelFn fused_chunks() { return sp_fused_kernel<4>; }
} // namespace spd
