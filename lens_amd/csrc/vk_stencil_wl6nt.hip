// Lag-1 wave-tile stencil (6 rows prefetched) with streaming stores: variant 6.
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <utility>

#include "vk_internal.h"
#include "vk_stencil_launch.h"

#define VK_WL_NT_STORE 1
#define VK_NT_NS vk_nt
#include "vk_stencil_nt.inc"

void vk_launch_wl6nt(VK_STENCIL_LAUNCH_ARGS) {
    if (k == 7)
        vk_nt::launch<7, 6>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
    else if (k == 9)
        vk_nt::launch<9, 6>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
    else if (k == 11)
        vk_nt::launch<11, 6>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
    else if (k == 10)   // the exact mode's 10-deep whole-step plan: 160 VGPRs (final pass: 178); PD is a
                        // multiple of 3 (the slot roles rotate with period 3)
        vk_nt::launch<10, 3>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
}
