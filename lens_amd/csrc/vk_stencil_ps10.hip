// Pair-sum tolerance-mode passes (vk_stencil_ps.h): the 10-deep pass of the
// C4 whole-step plan (variant 20), its own unit so that it compiles beside the others.
#include "vk_stencil_ps.h"

void vk_launch_ps10(VK_STENCIL_LAUNCH_ARGS) {
    (void)f0; (void)k;
    vk_ps::launch<10, 4, 2>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
}
