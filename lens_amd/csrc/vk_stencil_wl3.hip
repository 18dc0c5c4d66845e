// Lag-1 wave-tile stencil launchers, one prefetch depth per translation unit.
#include "vk_stencil_kernels.h"

namespace {

template <int K, int PD>
static void launch_wl(hipStream_t st, const double *src, double *dst, const double *f0, int nf, int64_t fs,
                      int ny, int out_lo, int out_hi, int in_lo, int in_hi, int top, int bot, double coef,
                      const double *mm, const VkPsCouple *cp) {
    VkPsCouple none = {};
    const VkPsCouple &c = cp ? *cp : none;
    constexpr int KH = K + (K & 1);
    constexpr int W = WT_COLS - 2 * KH;
    const int tiles_x = (ny + W - 1) / W;
    const int rch = chunk_rows(out_hi - out_lo, tiles_x, nf);
    const int chunks_y = (out_hi - out_lo + rch - 1) / rch;
    const int waves = tiles_x * chunks_y * nf;
    int ea = 0, eb = 0;
    vk_edge_chunks(K, out_lo, out_hi, rch, chunks_y, top, bot, ea, eb);
    if (f0)
        hipLaunchKernelGGL((k_diffuse_wl<K, PD, true>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst, f0, fs,
                           ny, out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef, mm, c, ea, eb);
    else
        hipLaunchKernelGGL((k_diffuse_wl<K, PD, false>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst, f0, fs,
                           ny, out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef, mm, c, ea, eb);
}

template <int PD>
static void launch_wl_k(int k, hipStream_t st, const double *src, double *dst, const double *f0, int nf,
                        int64_t fs, int ny, int out_lo, int out_hi, int in_lo, int in_hi, int top, int bot,
                        double coef, const double *mm, const VkPsCouple *cp) {
#define VK_WL(KC) case KC: launch_wl<KC, PD>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp); break
    switch (k) {
        VK_WL(3); VK_WL(5); VK_WL(7); VK_WL(9); VK_WL(11); VK_WL(13); VK_WL(15);
        default: break;
    }
#undef VK_WL
}

}  // namespace

void vk_launch_wl3(VK_STENCIL_LAUNCH_ARGS) {
    launch_wl_k<3>(k, st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp);
}
