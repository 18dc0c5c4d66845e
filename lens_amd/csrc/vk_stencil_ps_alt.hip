// Pair-sum tolerance-mode passes (vk_stencil_ps.h): A/B alternates at the C4
// depths 9 / 10 -- variant 21 = 2 rows prefetched, 22 = 6 rows prefetched,
// 23 = variant 20 with the chunk grid of odd tile columns staggered by half a chunk,
// 24 = variant 20 with plain (cached) stores, 25 = with streaming loads; 26 / 27 = variants
// 24 / 20 run one plane at a time (vk_diffuse: a plane's passes back to back, so the
// plane a pass writes -- 134 MB at C4 -- can stay in the 256-MB MALL for the next pass);
// 30-32 = the stage-0 ring held as 16-B vectors (vk_stencil_ps.h PsState), 4 / 6 / 2 rows prefetched.
#include "vk_stencil_ps.h"

void vk_launch_ps_alt(int variant, VK_STENCIL_LAUNCH_ARGS) {
    (void)f0;
#define VK_PSA(KC, PDC, CPC) \
    vk_ps::launch<KC, PDC, 2, CPC>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp)
    if (variant == 21 && k == 9) VK_PSA(9, 2, 0);
    else if (variant == 21 && k == 10) VK_PSA(10, 2, 0);
    else if (variant == 22 && k == 9) VK_PSA(9, 6, 0);
    else if (variant == 22 && k == 10) VK_PSA(10, 6, 0);
    // (variant 23 = variant 20's kernels with g_stencil_stagger set, vk_set_stencil_kernel)
    else if ((variant == 24 || variant == 26) && k == 10) VK_PSA(10, 4, 2);
    else if (variant == 25 && k == 10) VK_PSA(10, 4, 1);
    // 30 / 31 / 32: the stage-0 ring as 16-B vectors (no group-end drain), 4 / 6 / 2 rows prefetched
    else if (variant == 30 && k == 10) VK_PSA(10, 4, 4);
    else if (variant == 30 && k == 9) VK_PSA(9, 4, 4);
    else if (variant == 31 && k == 10) VK_PSA(10, 6, 4);
    else if (variant == 32 && k == 10) VK_PSA(10, 2, 4);
    else if (k == 10) vk_launch_ps10(k, st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
    else vk_launch_ps(k, st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
#undef VK_PSA
}
