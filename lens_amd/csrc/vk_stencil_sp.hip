// Stage-split pair-sum pass (vk_stencil_sp.h), variant 40: the 10-deep
// tolerance-mode pass with its stages spread over a workgroup's 5 waves.  It is
// the row-band default (multi-GPU C4: a middle rank's 100-substep step at N = 8 /
// 4 / 2 in 0.335 / 0.499 / 0.792 ms against 0.372 / 0.544 / 0.884 with variant
// 20, profiles/r05/r05fg/); on the whole 4096^2 plane variant 20 stays ahead
// (1.41-1.52 against 1.41-1.43 ms per 100 substeps, profiles/r05/r05b-r05e).
// Other depths, and passes that carry the agent coupling, run variant 20.
// Retired after their A/B (profiles/r05/): 41 (2 waves), 42 / 43 (4 columns per
// lane), 44-46 (8 / 12 / 16 rows prefetched by wave 0), 47 (one stage per wave),
// 48-51 (an LDS ring guarded by counters instead of the barrier).
#include "vk_stencil_sp.h"

// Rows per workgroup chunk (auto): by the rows the pass writes -- the fastest of
// 32-128 for a middle rank's band at N = 8 / 4 / 2 (profiles/r05/r05fg/).
static int sp_auto_rows(int out_rows) { return out_rows >= 1800 ? 64 : (out_rows >= 900 ? 96 : 48); }

bool vk_launch_sp(int variant, VK_STENCIL_LAUNCH_ARGS) {
    (void)f0;
    if (variant != 40 || k != 10 || (cp && cp->mode)) return false;
    const int rows = g_stencil_rows > 0 ? g_stencil_rows : sp_auto_rows(out_hi - out_lo);
    vk_sp::launch<10, 4, 2, 5>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, rows);
    return true;
}
