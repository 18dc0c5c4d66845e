// Stage-split pair-sum passes (vk_stencil_sp.h): variants 40-51, the 10-deep
// tolerance-mode pass of the C4 whole-step plan.  Other depths, and passes that
// carry the agent coupling, run variant 20 (vk_launch_ps_alt).  The variants are
// instantiated in vk_stencil_sp40..50.hip.
#include "vk_stencil_launch.h"

#define VK_SP_DECL(V) void vk_sp_launch_##V(VK_STENCIL_LAUNCH_ARGS, int rows);
VK_SP_DECL(40) VK_SP_DECL(41) VK_SP_DECL(42) VK_SP_DECL(43) VK_SP_DECL(44) VK_SP_DECL(45)
VK_SP_DECL(46) VK_SP_DECL(47) VK_SP_DECL(48) VK_SP_DECL(49) VK_SP_DECL(50) VK_SP_DECL(51)
#undef VK_SP_DECL

// rows per chunk = g_stencil_rows (0: 96)
bool vk_launch_sp(int variant, VK_STENCIL_LAUNCH_ARGS) {
    if (k != 10 || (cp && cp->mode)) return false;
    const int rows = g_stencil_rows > 0 ? g_stencil_rows : 96;
#define VK_SP_CASE(V) \
    case V: vk_sp_launch_##V(k, st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm, cp, rows); return true
    switch (variant) {
        VK_SP_CASE(40); VK_SP_CASE(41); VK_SP_CASE(42); VK_SP_CASE(43); VK_SP_CASE(44); VK_SP_CASE(45);
        VK_SP_CASE(46); VK_SP_CASE(47); VK_SP_CASE(48); VK_SP_CASE(49); VK_SP_CASE(50); VK_SP_CASE(51);
        default: return false;
    }
#undef VK_SP_CASE
}
