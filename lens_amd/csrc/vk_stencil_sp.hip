// Stage-split pair-sum passes (vk_stencil_sp.h): variant 40 and its A/B shapes, the
// 10-deep tolerance-mode pass of the C4 whole-step plan.  Other depths, and passes
// that carry the agent coupling, run variant 20 (vk_launch_ps_alt).
#include "vk_stencil_sp.h"

// variant -> (columns per lane C, waves per workgroup NW); rows per chunk = g_stencil_rows
// (0: 128)
bool vk_launch_sp(int variant, VK_STENCIL_LAUNCH_ARGS) {
    (void)f0;
    if (k != 10 || (cp && cp->mode)) return false;
    const int rows = g_stencil_rows > 0 ? g_stencil_rows : 128;
    switch (variant) {
        case 40: vk_sp::launch<10, 4, 2, 5>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, rows); return true;
        case 41: vk_sp::launch<10, 4, 2, 2>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, rows); return true;
        case 42: vk_sp::launch<10, 4, 4, 5>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, rows); return true;
        case 43: vk_sp::launch<10, 4, 4, 2>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, rows); return true;
        // deeper row prefetch in wave 0 (its iterations are ~5x shorter than a variant-20 wave's)
        case 44: vk_sp::launch<10, 8, 2, 5>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, rows); return true;
        case 45: vk_sp::launch<10, 12, 2, 5>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, rows); return true;
        case 46: vk_sp::launch<10, 16, 2, 5>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, rows); return true;
        case 47: vk_sp::launch<10, 12, 2, 10>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, rows); return true;
        default: return false;
    }
}
