// Pair-sum tolerance-mode passes (vk_stencil_ps.h): A/B alternates at the C4
// depths 9 / 10 -- variant 21 = 2 rows prefetched, 22 = 6 rows prefetched,
// 23 = variant 20 with the chunk grid of odd tile columns staggered by half a chunk,
// 24 = variant 20 with plain (cached) stores, 25 = with streaming loads.
#include "vk_stencil_ps.h"

void vk_launch_ps_alt(int variant, VK_STENCIL_LAUNCH_ARGS) {
    (void)f0;
#define VK_PSA(KC, PDC) vk_ps::launch<KC, PDC, 2>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm)
    if (variant == 21 && k == 9) VK_PSA(9, 2);
    else if (variant == 21 && k == 10) VK_PSA(10, 2);
    else if (variant == 22 && k == 9) VK_PSA(9, 6);
    else if (variant == 22 && k == 10) VK_PSA(10, 6);
    // (variant 23 = variant 20's kernels with g_stencil_stagger set, vk_set_stencil_kernel)
    else if (variant == 24 && k == 10)
        vk_ps::launch<10, 4, 2, 2>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm);
    else if (variant == 25 && k == 10)
        vk_ps::launch<10, 4, 2, 1>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm);
    else if (k == 10) vk_launch_ps10(k, st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm);
    else vk_launch_ps(k, st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm);
#undef VK_PSA
}
