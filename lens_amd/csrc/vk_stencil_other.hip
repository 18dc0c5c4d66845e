// Stencil launcher: workgroup tile with LDS neighbour exchange (variant 0).
#include "vk_stencil_kernels.h"

namespace {

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

void vk_launch_tb(VK_STENCIL_LAUNCH_ARGS) {
    launch_tb_k(k, st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm);
}
