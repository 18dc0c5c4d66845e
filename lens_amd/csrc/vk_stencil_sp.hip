// Stage-split pair-sum pass (vk_stencil_sp.h), variant 40: the 10-deep
// tolerance-mode pass with its stages spread over a workgroup's 5 waves.  It is
// the row-band default (multi-GPU C4: a middle rank's 100-substep step at N = 8 /
// 4 / 2 in 0.335 / 0.499 / 0.792 ms against 0.372 / 0.544 / 0.884 with variant
// 20, profiles/r05/r05fg/) and C3's (1024^2: 0.222 against 0.320 ms per step,
// profiles/r05/r05q/); on the whole 4096^2 plane it ties variant 20 (1.384 against
// 1.390 ms per 100 substeps at 86-row chunks, profiles/r05/r05r/).
// Other depths, and passes that carry the agent coupling, run variant 20.
// Retired after their A/B (profiles/r05/): 41 (2 waves), 42 / 43 (4 columns per
// lane), 44-46 (8 / 12 / 16 rows prefetched by wave 0), 47 (one stage per wave),
// 48-51 (an LDS ring guarded by counters instead of the barrier).
#include "vk_stencil_sp.h"

bool vk_launch_sp(int variant, VK_STENCIL_LAUNCH_ARGS) {
    (void)f0;
    if (variant != 40 || k != 10 || (cp && cp->mode)) return false;
    const int rows = g_stencil_rows > 0 ? g_stencil_rows : 0;   // 0: whole rounds of workgroups (vk_sp::round_rows)
    vk_sp::launch<10, 4, 2, 5>(st, src, dst, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, rows);
    return true;
}
