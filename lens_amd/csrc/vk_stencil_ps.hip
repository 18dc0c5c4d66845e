// Pair-sum tolerance-mode passes (vk_stencil_ps.h): the default variant 20.
#include "vk_stencil_ps.h"
#include "vk_internal.h"

// variant 20: 2 columns per lane, 4 rows prefetched
void vk_launch_ps(VK_STENCIL_LAUNCH_ARGS) {
    (void)f0;   // the tolerance mode's final pass writes the new field as is
#define VK_PS(KC) case KC: vk_ps::launch<KC, 4, 2>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp); break
    switch (k) {
        VK_PS(3); VK_PS(5); VK_PS(7); VK_PS(9); VK_PS(11);
        default: vk::set_error("vk_launch_ps: no pair-sum pass of depth %d", k); break;
    }
#undef VK_PS
}
