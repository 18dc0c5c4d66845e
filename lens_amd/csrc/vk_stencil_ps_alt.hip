// Pair-sum tolerance-mode passes (vk_stencil_ps.h): variant 30, the stage-0 ring
// held as 16-B vectors (no drain of the load queue at the end of each unrolled
// group), at the C4 depths 9 / 10; every other variant / depth runs variant 20.
// Retired after their A/B (profiles/r04/r04a, r04f, r04i): 21 / 22
// (2 / 6 rows prefetched), 23 (half-chunk stagger of odd tile columns), 24 / 25
// (cached stores / streaming loads), 26 / 27 (one plane at a time), 28 / 29 (coupled
// gather after the stencil, cached final pass), 31 / 32 (vector ring, 6 / 2 rows);
// for row bands (profiles/r04/r04q-r04u): 34 (cached stores + vector ring), 37 (the
// general body on every tile), 38 / 39 (8 / 12 rows prefetched) -- 33 (cached
// stores) became the 10-deep pass's rule for MALL-sized passes (vk_stencil_ps10.hip).
#include "vk_stencil_ps.h"

void vk_launch_ps_alt(int variant, VK_STENCIL_LAUNCH_ARGS) {
    (void)f0;
    if (variant == 30 && k == 10)
        vk_ps::launch<10, 4, 2, 4>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
    else if (variant == 30 && k == 9)
        vk_ps::launch<9, 4, 2, 4>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
    else if (k == 10) vk_launch_ps10(k, st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
    else vk_launch_ps(k, st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
}
