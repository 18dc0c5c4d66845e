// Launchers of the fused-pass stencil kernels (vk_stencil_*.hip), called by
// vk_diffuse (vk_lattice.hip).  k = substeps fused in the pass (odd, 3..15);
// f0 != nullptr marks the FINAL pass (writes f0 + (f - f0)).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define VK_STENCIL_LAUNCH_ARGS                                                                                 \
    int k, hipStream_t st, const double *src, double *dst, const double *f0, int nf, int64_t fs, int ny,        \
        int out_lo, int out_hi, int in_lo, int in_hi, int top, int bot, double coef, const double *mm

extern int g_stencil_rows;   // output rows per wave tile, 0 = auto (vk_lattice.hip, vk_set_stencil_kernel)
extern int g_stencil_mode;   // 0 = bit-exact (default), 1 = tolerance / FMA (vk_set_stencil_mode)
extern int g_stencil_stagger;  // pair-sum passes: odd tile columns' chunk grid shifted by half a chunk (variant 23)

void vk_launch_wl3(VK_STENCIL_LAUNCH_ARGS);          // lag-1 wave tile, 3 rows prefetched
void vk_launch_wl6(VK_STENCIL_LAUNCH_ARGS);          // lag-1 wave tile, 6 rows prefetched
void vk_launch_wl6nt(VK_STENCIL_LAUNCH_ARGS);        // as wl6 with streaming stores (k = 7, 9, 11; 10 tolerance mode)
// Agent coupling carried by a pair-sum pass (vk_diffuse_coupled): each wave
// handles the agents whose bins lie in its own output rows x columns.  Agents
// are stored in bin order (bins ascending); seg[r * nseg + s] = the first agent
// with bin >= r * ny + 16 s.
#define VK_COUPLE_MAX_FIELDS 8
struct VkPsCouple {
    const int32_t *bins;
    const int32_t *seg;
    int32_t nseg;
    int32_t n;                             // agents
    int32_t mode;                          // bit 0: gather before the pass, bit 1: exchange after it
    double *gdst;                          // gather: gdst[grow[f] * gld + a] = plane f at bins[a] (pre-pass)
    int64_t gld;
    const int64_t *counts;                 // exchange: plane f += counts[crow[f] * cld + a] / bva * 1000
    int64_t cld;
    double bva;
    int8_t grow[VK_COUPLE_MAX_FIELDS];     // -1 = none
    int8_t crow[VK_COUPLE_MAX_FIELDS];
};

void vk_launch_ps(VK_STENCIL_LAUNCH_ARGS, const VkPsCouple *cp);     // tolerance mode, pair-sum form (k = 3, 5, 7, 9, 11)
void vk_launch_ps10(VK_STENCIL_LAUNCH_ARGS, const VkPsCouple *cp);   // the same, k = 10
// variant 20-25 dispatch (21-25: A/B alternates); cp (nullable) = agent coupling
void vk_launch_ps_alt(int variant, VK_STENCIL_LAUNCH_ARGS, const VkPsCouple *cp = nullptr);
