// The 10-deep pair-sum pass with the vertical stash (variant 60..62, vk_stencil_ps.h
// PsStash): 4 vertically adjacent chunks per workgroup, the shared boundary rows handed
// up through LDS instead of read twice.  Its own unit so that it compiles beside the others.
#include "vk_stencil_ps.h"

// Not taken (false) unless every chunk is 64 rows.
// variant: 60 = 16 stash rows, XCD windows of 4 groups; 61 = 16 rows, windows of 8;
// 62 = 17 rows (the most 3 workgroups per CU hold in 160 KB of LDS), windows of 4;
// A/B only: 63 = variant 60's groups without stash reads, 64 = variant 20's tile order
// through the same code
bool vk_launch_ps10_vs(int variant, VK_STENCIL_LAUNCH_ARGS) {
    (void)f0; (void)k;
    switch (variant) {
        case 60: return vk_ps::launch_vs<10, 4, 2, 16, 4>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
        case 61: return vk_ps::launch_vs<10, 4, 2, 16, 8>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
        case 62: return vk_ps::launch_vs<10, 4, 2, 17, 4>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
        case 63: return vk_ps::launch_vs<10, 4, 2, 16, 4, 1>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
        case 64: return vk_ps::launch_vs<10, 4, 2, 16, 4, 2>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
        default: return false;
    }
}
