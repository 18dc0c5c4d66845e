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

void vk_launch_wl3(VK_STENCIL_LAUNCH_ARGS);          // lag-1 wave tile, 3 rows prefetched
void vk_launch_wl6(VK_STENCIL_LAUNCH_ARGS);          // lag-1 wave tile, 6 rows prefetched
void vk_launch_wl9(VK_STENCIL_LAUNCH_ARGS);          // lag-1 wave tile, 9 rows prefetched
void vk_launch_wl6nt(VK_STENCIL_LAUNCH_ARGS);        // as wl6 with streaming stores (k = 7, 9, 11)
void vk_launch_wl6r(VK_STENCIL_LAUNCH_ARGS);         // wl6nt, stage 0 on the prefetch ring (k = 7, 9, 11)
void vk_launch_wl6b(VK_STENCIL_LAUNCH_ARGS);         // wl6r with branch-free buffer stores (k = 7, 9, 11)
void vk_launch_wl3b(VK_STENCIL_LAUNCH_ARGS);         // wl6b with 3 rows of lookahead (k = 7, 9, 11)
void vk_launch_wl6z(VK_STENCIL_LAUNCH_ARGS);
void vk_launch_wl6nt10p6(VK_STENCIL_LAUNCH_ARGS);   // 10-deep fma pass, 6 rows prefetched (variant 16)         // wl6nt with zigzag chunks (k = 7, 9, 11)
void vk_launch_tb(VK_STENCIL_LAUNCH_ARGS);           // workgroup tile, LDS neighbour exchange
