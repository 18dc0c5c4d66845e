// Pair-sum tolerance-mode passes (vk_stencil_ps.h): the 10-deep pass of the
// C4 whole-step plan (variant 20), its own unit so that it compiles beside the others.
#include "vk_stencil_ps.h"

// A pass whose planes fit the 256 MB MALL twice over (source + destination rows
// <= 192 MB: a row band at N >= 4 on 4096^2 x 2) stores through the caches, so
// the next pass finds its rows there: a middle rank's step at N = 8 / 4 runs
// 0.377 / 0.574 ms against 0.391 / 0.586 with streaming stores, while the whole
// plane (537 MB per pass) is 8 % slower with cached stores
// (profiles/r04/r04q_rank8.log, r04t_rank8.log, r04u_rank4.log).
void vk_launch_ps10(VK_STENCIL_LAUNCH_ARGS) {
    (void)f0; (void)k;
    const double pass_bytes = 16.0 * (double)(in_hi - in_lo) * (double)ny * (double)nf;
    if (pass_bytes <= 192.0 * 1024 * 1024)
        vk_ps::launch<10, 4, 2, 2>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
    else
        vk_ps::launch<10, 4, 2>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
}

// Both edge strips of a band's 10-deep pass in one launch (vk_diffuse_part): rows
// [out_lo, out_hi) without [gap_lo, gap_hi).  The strips are a few dozen rows each,
// so a pass is latency-bound, and one launch costs about what one strip did.
void vk_launch_ps10_strips(VK_STENCIL_LAUNCH_ARGS, int gap_lo, int gap_hi) {
    (void)f0; (void)k;
    vk_ps::launch<10, 4, 2, 2>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp, gap_lo,
                               gap_hi);
}

// Variant 70: 16 halo columns per side and 96 written columns, so every tile's loads
// and stores cover whole 128-B lines (variant 20: 10 and 108, a row's 864-B store
// shares its end lines with the next tile's).  12 % more VALU per written cell, but
// the C4 step's passes take 1.160 against 1.188 ms (profiles/r06/r06l/); the same
// store-policy rule as vk_launch_ps10.
void vk_launch_ps10_aligned(VK_STENCIL_LAUNCH_ARGS) {
    (void)f0; (void)k;
    const double pass_bytes = 16.0 * (double)(in_hi - in_lo) * (double)ny * (double)nf;
    if (pass_bytes <= 192.0 * 1024 * 1024)
        vk_ps::launch<10, 4, 2, 2, 16>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
    else
        vk_ps::launch<10, 4, 2, 0, 16>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
}
