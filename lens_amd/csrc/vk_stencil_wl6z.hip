// Lag-1 wave-tile stencil (6 rows prefetched) with streaming stores, zigzag chunks
// (VK_WL_ZIGZAG in vk_stencil_kernels.h: odd chunks walked bottom-up in the
// tolerance mode, workgroups down a column tile): variant 15.
#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <utility>

#include "vk_internal.h"
#include "vk_stencil_launch.h"

#define VK_WL_NT_STORE 1
#define VK_WL_ZIGZAG 1
#define VK_NT_NS vk_nz
#include "vk_stencil_nt.inc"

void vk_launch_wl6z(VK_STENCIL_LAUNCH_ARGS) {
    if (k == 7)
        vk_nz::launch<7, 6>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm);
    else if (k == 9)
        vk_nz::launch<9, 6>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm);
    else if (k == 11)
        vk_nz::launch<11, 6>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm);
}
