// Lag-1 wave-tile stencil (3 rows prefetched) with streaming stores: variant 14
// = variant 13 with a 3-row lookahead: ring of 6, unrolled by 6 (variant 6's code size), with
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
#define VK_NT_NS vk_n3
#include "vk_stencil_nt.inc"

void vk_launch_wl3b(VK_STENCIL_LAUNCH_ARGS) {
    if (k == 7)
        vk_n3::launch<7, 3>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm);
    else if (k == 9)
        vk_n3::launch<9, 3>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm);
    else if (k == 11)
        vk_n3::launch<11, 3>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm);
}
