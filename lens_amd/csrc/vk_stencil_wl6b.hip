// Lag-1 wave-tile stencil (6 rows prefetched) with streaming stores: variant 13
// = variant 6's body with stage 0 reading the prefetch ring (VK_WL_RING) and
// branch-free buffer stores (VK_WL_BUF_STORE), vk_stencil_kernels.h.
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <utility>

#include "vk_internal.h"
#include "vk_stencil_launch.h"

#define VK_WL_NT_STORE 1
#define VK_WL_RING 1
#define VK_WL_BUF_STORE 1
#define VK_NT_NS vk_nb
#include "vk_stencil_nt.inc"

void vk_launch_wl6b(VK_STENCIL_LAUNCH_ARGS) {
    if (k == 7)
        vk_nb::launch<7, 6>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm);
    else if (k == 9)
        vk_nb::launch<9, 6>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm);
    else if (k == 11)
        vk_nb::launch<11, 6>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm);
}
