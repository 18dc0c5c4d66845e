// Stencil launchers: lag-2 wave tile, workgroup/LDS tile, occupancy-capped lag-1 tile.
#include "vk_stencil_kernels.h"

namespace {

template <int K, int PD>
static void launch_wl4(hipStream_t st, const double *src, double *dst, const double *f0, int nf, int64_t fs,
                       int ny, int out_lo, int out_hi, int in_lo, int in_hi, int top, int bot, double coef,
                       const double *mm) {
    constexpr int KH = K + (K & 1);
    constexpr int W = WT_COLS - 2 * KH;
    const int tiles_x = (ny + W - 1) / W;
    const int rch = chunk_rows(out_hi - out_lo, tiles_x, nf);
    const int chunks_y = (out_hi - out_lo + rch - 1) / rch;
    const int waves = tiles_x * chunks_y * nf;
    if (f0)
        hipLaunchKernelGGL((k_diffuse_wl4<K, 3, true>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst, f0, fs,
                           ny, out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef, mm);
    else
        hipLaunchKernelGGL((k_diffuse_wl4<K, PD, false>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst, f0, fs,
                           ny, out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef, mm);
}

static void launch_wt_k(int k, hipStream_t st, const double *src, double *dst, const double *f0, int nf,
                        int64_t fs, int ny, int out_lo, int out_hi, int in_lo, int in_hi, int top, int bot,
                        double coef, const double *mm) {
#define VK_WT(KC) case KC: launch_wt<KC>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm); break
    switch (k) {
        VK_WT(3); VK_WT(5); VK_WT(7); VK_WT(9); VK_WT(11); VK_WT(13); VK_WT(15);
        default: break;
    }
#undef VK_WT
}

template <int K>
static void launch_tb(hipStream_t st, const double *src, double *dst, const double *f0, int nf,
                      int64_t fs, int ny, int out_lo, int out_hi, int in_lo, int in_hi, int top, int bot,
                      double coef, const double *mm) {
    const int rch = 128;
    dim3 grid((ny + (TB_BX - 2 * K) - 1) / (TB_BX - 2 * K), (out_hi - out_lo + rch - 1) / rch, nf);
    hipLaunchKernelGGL(k_diffuse_tb<K>, grid, dim3(TB_BX), 0, st, src, dst, f0, fs, ny, out_lo, out_hi, in_lo,
                       in_hi, top, bot, rch, coef, mm);
}

static void launch_tb_k(int k, hipStream_t st, const double *src, double *dst, const double *f0, int nf,
                        int64_t fs, int ny, int out_lo, int out_hi, int in_lo, int in_hi, int top, int bot,
                        double coef, const double *mm) {
#define VK_TB(KC) case KC: launch_tb<KC>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm); break
    switch (k) {  // odd depths only (see vk_diffuse)
        VK_TB(3); VK_TB(5); VK_TB(7); VK_TB(9); VK_TB(11); VK_TB(13); VK_TB(15);
        default: break;
    }
#undef VK_TB
}

}  // namespace

void vk_launch_wt(VK_STENCIL_LAUNCH_ARGS) {
    launch_wt_k(k, st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm);
}

void vk_launch_tb(VK_STENCIL_LAUNCH_ARGS) {
    launch_tb_k(k, st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm);
}

void vk_launch_wl4(VK_STENCIL_LAUNCH_ARGS) {
    if (k == 7)
        launch_wl4<7, 6>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm);
    else if (k == 9)
        launch_wl4<9, 6>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm);
}
