// Lag-1 wave tile at 4 waves per SIMD (variant 9).
//
// The stencil pass is issue-latency bound: each stage is a chain of six
// dependent FP64 operations, and one wave issues well below the SIMD's rate,
// so throughput comes from the number of resident waves.  k_diffuse_wl needs
// ~92 live VGPRs in its steady state at depth 9, but its boundary-tile body
// (clamped scalar loads, per-column reflect selects) and its 6-row prefetch
// push the kernel to 158 VGPRs = 3 waves/SIMD.  This variant keeps one body
// for all tiles:
//   * boundary columns load the same 16-byte pair as interior ones, at a
//     clamped pair index (lanes outside the plane read a valid pair; their
//     values never reach a written column, because column 0 and column ny-1
//     reflect onto themselves);
//   * the only column selects left are at column 0 (an A column: tiles start
//     at even columns) and column ny-1 (a B column: ny is even here), as
//     lane masks; the row reflects are wave-uniform;
//   * 3 rows of prefetch;
// so the whole kernel fits 128 VGPRs (amdgpu_waves_per_eu(4)).  Odd-width
// planes take variant 6.  Same arithmetic in the same order: bit-identical.
#define VK_WL_NT_STORE 1
#include "vk_stencil_kernels.h"

namespace {

struct WcLane {
    int cA;          // this lane's first column (x0 - KH + 2*lane), may lie outside [0, ny)
    int cP;          // the clamped, even pair index it loads
    int ny;
    bool w;          // writes its pair
    bool l0, rN;     // column 0 is its A column / column ny-1 is its B column
};

__device__ __forceinline__ double2 wc_load(const double *__restrict__ p, int64_t row_off, const WcLane &L) {
    return *reinterpret_cast<const double2 *>(p + row_off + L.cP);
}

template <int K, int PD, bool EDGE, bool FINAL, bool STEADY, int U>
__device__ __forceinline__ void wc_iter(double2 (&S0)[K], double2 (&S1)[K], double2 (&S2)[K], double2 (&pf)[PD],
                                        double2 (&gp)[3], const double *__restrict__ s, double *d, const double *g,
                                        const WcLane &L, int i, int c0, int c1, int in_lo, int in_hi,
                                        int top_reflect, int bot_reflect, double coef) {
    constexpr int R = U % 3;
    double2(&UP)[K] = R == 0 ? S0 : (R == 1 ? S1 : S2);
    double2(&CN)[K] = R == 0 ? S1 : (R == 1 ? S2 : S0);
    double2(&FR)[K] = R == 0 ? S2 : (R == 1 ? S0 : S1);
    const int64_t ny = L.ny;
    FR[0] = pf[U];                                                                  // row i
    pf[U] = wc_load(s, (int64_t)min(max(i + PD, in_lo), in_hi - 1) * ny, L);     // row i+PD
    const int r_out = i - K;
    const bool row_ok = STEADY || (r_out >= c0 && r_out < c1);
    double2 base = make_double2(0.0, 0.0);
    if (FINAL) {   // base row r_out arrived 3 iterations ago; fetch row r_out+3 (clamped into the chunk)
        base = gp[R];
        gp[R] = wc_load(g, (int64_t)min(max(r_out + 3, c0), c1 - 1) * ny, L);
    }
#pragma unroll
    for (int q = 0; q < K; ++q) {
        if (!STEADY && (i < c0 - K + 2 + 2 * q || i >= c1 + K)) continue;
        const int r = i - 1 - q;
        const double2 cen = CN[q];
        double2 up = UP[q], dn = FR[q];
        if (EDGE) {   // wave-uniform
            if (r == top_reflect) up = cen;
            if (r == bot_reflect) dn = cen;
        }
        double leftA = dpp_from_lane_below(cen.y), rightB = dpp_from_lane_above(cen.x);
        if (EDGE) {
            leftA = L.l0 ? cen.x : leftA;
            rightB = L.rN ? cen.y : rightB;
        }
        const double lapA = ((fma(-4.0, cen.x, up.x + leftA)) + cen.y) + dn.x;
        const double lapB = ((fma(-4.0, cen.y, up.y + cen.x)) + rightB) + dn.y;
        double2 v = make_double2(cen.x + coef * lapA, cen.y + coef * lapB);
        if (q + 1 < K) {
            FR[q + 1] = v;
        } else if (row_ok) {
            if (FINAL) v = make_double2(base.x + (v.x - base.x), base.y + (v.y - base.y));
            if (L.w) wl_store(d + (int64_t)r_out * ny + L.cA, v);
        }
    }
}

template <int K, int PD, bool EDGE, bool FINAL, bool STEADY, int U0, int... Us>
__device__ __forceinline__ void wc_group(double2 (&S0)[K], double2 (&S1)[K], double2 (&S2)[K], double2 (&pf)[PD],
                                         double2 (&gp)[3], const double *__restrict__ s, double *d, const double *g,
                                         const WcLane &L, int i, int c0, int c1, int in_lo, int in_hi,
                                         int top_reflect, int bot_reflect, double coef) {
    wc_iter<K, PD, EDGE, FINAL, STEADY, U0>(S0, S1, S2, pf, gp, s, d, g, L, i, c0, c1, in_lo, in_hi, top_reflect,
                                            bot_reflect, coef);
    if constexpr (sizeof...(Us) > 0)
        wc_group<K, PD, EDGE, FINAL, STEADY, Us...>(S0, S1, S2, pf, gp, s, d, g, L, i + 1, c0, c1, in_lo, in_hi,
                                                    top_reflect, bot_reflect, coef);
}

template <int K, int PD, bool EDGE, bool FINAL, int... Us>
__device__ __forceinline__ void wc_body(std::integer_sequence<int, Us...>, const double *__restrict__ s, double *d,
                                        const double *g, const WcLane &L, int c0, int c1, int in_lo, int in_hi,
                                        int top_reflect, int bot_reflect, double coef) {
    double2 S0[K], S1[K], S2[K], pf[PD], gp[3];
#pragma unroll
    for (int q = 0; q < K; ++q) S0[q] = S1[q] = S2[q] = make_double2(0.0, 0.0);
    const int64_t ny = L.ny;
    const int i0 = c0 - K + 2, i1 = c1 + K;          // iterations [i0, i1)
    const int s_lo = c0 + K, s_hi = c1 + K - 1;      // every stage active for i in [s_lo, s_hi]
    S0[0] = wc_load(s, (int64_t)min(max(i0 - 2, in_lo), in_hi - 1) * ny, L);
    S1[0] = wc_load(s, (int64_t)min(max(i0 - 1, in_lo), in_hi - 1) * ny, L);
#pragma unroll
    for (int u = 0; u < PD; ++u) pf[u] = wc_load(s, (int64_t)min(max(i0 + u, in_lo), in_hi - 1) * ny, L);
#pragma unroll
    for (int u = 0; u < 3; ++u)
        gp[u] = FINAL ? wc_load(g, (int64_t)min(max(i0 - K + u, c0), c1 - 1) * ny, L) : make_double2(0.0, 0.0);
#define WC_ARGS S0, S1, S2, pf, gp, s, d, g, L, i, c0, c1, in_lo, in_hi, top_reflect, bot_reflect, coef
    int i = i0;
    for (; i + PD <= i1 && i < s_lo; i += PD) wc_group<K, PD, EDGE, FINAL, false, Us...>(WC_ARGS);   // fill
    for (; i + PD - 1 <= s_hi; i += PD) wc_group<K, PD, EDGE, FINAL, true, Us...>(WC_ARGS);          // steady
    for (; i + PD <= i1; i += PD) wc_group<K, PD, EDGE, FINAL, false, Us...>(WC_ARGS);               // drain
    ((i + Us < i1 ? wc_iter<K, PD, EDGE, FINAL, false, Us>(S0, S1, S2, pf, gp, s, d, g, L, i + Us, c0, c1, in_lo,
                                                           in_hi, top_reflect, bot_reflect, coef)
                  : void()),
     ...);
#undef WC_ARGS
}

template <int K, int PD, bool FINAL, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void k_diffuse_wlc(VK_WL_PARAMS) {
    constexpr int KH = K + (K & 1);
    constexpr int W = WT_COLS - 2 * KH;
    const int wave = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
    const int lane = threadIdx.x & 63;
    if (wave >= tiles_x * chunks_y * n_fields) return;
    const int tx = wave % tiles_x;
    const int ty = (wave / tiles_x) % chunks_y;
    const int f = wave / (tiles_x * chunks_y);
    if (uniform && uniform[2 * f] == uniform[2 * f + 1]) return;
    const int c0 = out_lo + ty * rows_per_chunk;
    const int c1 = min(c0 + rows_per_chunk, out_hi);
    const int x0 = tx * W;
    WcLane L;
    L.ny = ny;
    L.cA = x0 - KH + 2 * lane;
    L.cP = min(max(L.cA, 0), ny - 2);
    L.w = lane >= KH / 2 && lane < 64 - KH / 2 && L.cA < ny;
    L.l0 = L.cA == 0;
    L.rN = L.cA + 1 == ny - 1;
    const double *s = src + (int64_t)f * field_stride;
    double *d = dst + (int64_t)f * field_stride;
    const double *g = f0 ? f0 + (int64_t)f * field_stride : nullptr;
    const bool edge = (x0 - KH <= 0) || (x0 - KH + WT_COLS >= ny) ||
                      (top_reflect >= c0 - 2 * K - 2 && top_reflect <= c1 + 2 * K) ||
                      (bot_reflect >= c0 - 2 * K - 2 && bot_reflect <= c1 + 2 * K);
    if (edge)
        wc_body<K, PD, true, FINAL>(std::make_integer_sequence<int, PD>(), s, d, g, L, c0, c1, in_lo, in_hi,
                                    top_reflect, bot_reflect, coef);
    else
        wc_body<K, PD, false, FINAL>(std::make_integer_sequence<int, PD>(), s, d, g, L, c0, c1, in_lo, in_hi,
                                     top_reflect, bot_reflect, coef);
}

template <int K, int WPE>
void launch_wlc(hipStream_t st, const double *src, double *dst, const double *f0, int nf, int64_t fs, int ny,
                int out_lo, int out_hi, int in_lo, int in_hi, int top, int bot, double coef, const double *mm) {
    constexpr int KH = K + (K & 1);
    constexpr int W = WT_COLS - 2 * KH;
    const int tiles_x = (ny + W - 1) / W;
    const int rch = chunk_rows(out_hi - out_lo, tiles_x, nf);
    const int chunks_y = (out_hi - out_lo + rch - 1) / rch;
    const int waves = tiles_x * chunks_y * nf;
    if (f0)
        hipLaunchKernelGGL((k_diffuse_wlc<K, 3, true, WPE>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst, f0,
                           fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef, mm);
    else
        hipLaunchKernelGGL((k_diffuse_wlc<K, 3, false, WPE>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst,
                           f0, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef, mm);
}

}  // namespace

// ny must be even (the launcher in vk_lattice.hip routes odd widths elsewhere)
void vk_launch_wlc(VK_STENCIL_LAUNCH_ARGS) {
#define VK_WC(KC, WPE) \
    case KC: launch_wlc<KC, WPE>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm); break
    switch (k) {
        VK_WC(3, 4); VK_WC(5, 4); VK_WC(7, 4); VK_WC(9, 3); VK_WC(11, 3);
        default: break;
    }
#undef VK_WC
}
