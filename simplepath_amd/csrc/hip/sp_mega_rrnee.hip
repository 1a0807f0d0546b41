// sp_mega_rrnee.hip -- IterativeIntegratorRRNEE megakernel (lock-step samples, one lane per pixel).
// Multiple-importance estimates served across the wave (sp_path.hpp serve_rho).  With them, no
// RNG draw-ahead window and the estimate's words touched in advance (as in the DirectLighting
// megakernel): elf 1024^2 @ 16 spp 739-745 -> 746-757 Mrays/s (profiles/r03/ab_rrnee_served.txt).
#ifndef SP_SERVE_RHO
#define SP_SERVE_RHO 1
#endif
#define SP_RNG_PF 0
#define SP_RHO_TOUCH 1
// Twist ahead at the bounce start once within 144 words of the end (the blocked twist, batched
// over the wave), so the 140-word reservation of a served bounce (sp_path.hpp integrate_rrnee)
// never falls back to the compact per-lane twist: 793-797 -> 810-822 Mrays/s on elf 1024^2 @ 16 spp.
#define SP_RNG_MARGIN 144
// The bounce's own Material::sample estimate joins the first light's served round (sp_path.hpp
// integrate_rrnee): 768-775 -> 783-797 Mrays/s on elf 1024^2 @ 16 spp (profiles/r03/ab_rrnee_served.txt).
#ifndef SP_SERVE_SAMPLE
#define SP_SERVE_SAMPLE 1
#endif
// Served estimates read their owner's 32 words as one aligned 16-byte pair per sample whatever the
// parity (sp_path.hpp SP_RHO_ALIGNED): elf 1024^2 @ 16 spp 1067-1084 -> 1085-1098, its 8-way shard
// 1236-1243 -> 1253-1270 Mrays/s (profiles/r06/served/ab_aligned.log); the lanes' own estimates
// aligned too measured lower (1080-1092, 1250-1254), and paired draws with a single-load branch
// for odd positions lost (SP_SERVED_PAIR: 1039-1051, 1196-1199).
#ifndef SP_SERVED_ALIGNED
#define SP_SERVED_ALIGNED 1
#endif
// ... and without the LDS-DMA touch ahead of them (the owners' own estimates keep it): level on elf
// 1024^2 @ 16 spp (1080-1092 against 1084-1085), the 8-way shard 1254-1270 -> 1275 (ab_notouch.log)
#ifndef SP_SERVED_TOUCH
#define SP_SERVED_TOUCH 0
#endif
#include "sp_mega.hpp"

namespace spd {
KernelFn mega_rrnee(int w)
{
    // w = waves per SIMD (sp_render_tiles: 3 unless waves_per_simd or the LDS says otherwise);
    // elf 1024^2 x 16 spp: 476 / 553 / 519 Mrays/s at 2 / 3 / 4 waves (profiles/r02/s5).  Two
    // schedules that share estimates across lanes were exact but slower: one shared
    // estimate per wave round (455 vs 579 Mrays/s, profiles/r03) and estimates served block-wide
    // (311, profiles/r03/wprof_elf_1k_rrnee_block.txt).
    if (w == 2) return sp_render_kernel<SP_INTEGRATOR_ITERATIVE_RRNEE, 2>;
    if (w == 4) return sp_render_kernel<SP_INTEGRATOR_ITERATIVE_RRNEE, 4>;
    return sp_render_kernel<SP_INTEGRATOR_ITERATIVE_RRNEE, 3>;
}
} // namespace spd
