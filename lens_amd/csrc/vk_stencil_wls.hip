// Lag-1 wave tile, "split stage" form (variant 10).
//
// Same tile, lanes and arithmetic as variant 9, reordered: stage q's
// five-point sum for row r needs only one value it does not already hold at
// the end of the previous iteration -- the down neighbour, which stage q-1
// produces in this one.  So each stage carries T = ((up + left) + (-4 c)) +
// right, computed one iteration early from its centre row (DPP neighbours
// included), plus the centre c itself, and the in-iteration chain through the
// K stages is  lap = T + down; v = c + coef*lap  (3 dependent FP64 ops per
// stage instead of 6); the T of the next row is computed off that chain.  The
// per-stage state is two row pairs as before, but it is updated in place
// (no three-way register rotation), which keeps the allocation tight.
// Same operations on the same operands in the same order: bit-identical.
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
__device__ __forceinline__ void ws_iter(double2 (&T)[K], double2 (&C)[K], double2 (&pf)[PD], double2 (&gp)[3],
                                        const double *__restrict__ s, double *d, const double *g, const WcLane &L,
                                        int i, int c0, int c1, int in_lo, int in_hi, int top_reflect,
                                        int bot_reflect, double coef) {
    const int64_t ny = L.ny;
    double2 x = pf[U];                                                              // row i: stage 0's input
    pf[U] = wc_load(s, (int64_t)min(max(i + PD, in_lo), in_hi - 1) * ny, L);     // row i+PD
    const int r_out = i - K;
    const bool row_ok = STEADY || (r_out >= c0 && r_out < c1);
    double2 base = make_double2(0.0, 0.0);
    if (FINAL) {   // base row r_out arrived 3 iterations ago; fetch row r_out+3 (clamped into the chunk)
        base = gp[U % 3];
        gp[U % 3] = wc_load(g, (int64_t)min(max(r_out + 3, c0), c1 - 1) * ny, L);
    }
#pragma unroll
    for (int q = 0; q < K; ++q) {
        // stage q's input x is row i-q; it computes row i-1-q (valid once it has
        // seen two valid inputs) and folds x into T/C for row i-q
        const bool cmp = STEADY || (i >= c0 - K + 2 + 2 * q && i < c1 + K);
        const bool upd = STEADY || (i >= c0 - K + 2 * q && i < c1 + K);
        double2 v = make_double2(0.0, 0.0);
        if (cmp) {
            double2 dn = x;
            if (EDGE && i - 1 - q == bot_reflect) dn = C[q];
            v = make_double2(C[q].x + coef * (T[q].x + dn.x), C[q].y + coef * (T[q].y + dn.y));
        }
        if (upd) {
            double2 up = C[q];
            if (EDGE && i - q == top_reflect) up = x;
            double leftA = dpp_from_lane_below(x.y), rightB = dpp_from_lane_above(x.x);
            if (EDGE) {
                leftA = L.l0 ? x.x : leftA;
                rightB = L.rN ? x.y : rightB;
            }
            T[q] = make_double2((fma(-4.0, x.x, up.x + leftA)) + x.y, (fma(-4.0, x.y, up.y + x.x)) + rightB);
            C[q] = x;
            // pin the update here: left to itself the compiler sinks every stage's
            // update to the end of the iteration, which keeps K more rows live
            asm volatile("" : "+v"(T[q].x), "+v"(T[q].y));
        }   // keep stages apart: hoisting updates only lengthens live ranges
        if (q + 1 < K) {
            x = v;
        } else if (row_ok) {
            if (FINAL) v = make_double2(base.x + (v.x - base.x), base.y + (v.y - base.y));
            if (L.w) wl_store(d + (int64_t)r_out * ny + L.cA, v);
        }
    }
}

template <int K, int PD, bool EDGE, bool FINAL, bool STEADY, int U0, int... Us>
__device__ __forceinline__ void ws_group(double2 (&T)[K], double2 (&C)[K], double2 (&pf)[PD], double2 (&gp)[3],
                                         const double *__restrict__ s, double *d, const double *g, const WcLane &L,
                                         int i, int c0, int c1, int in_lo, int in_hi, int top_reflect,
                                         int bot_reflect, double coef) {
    ws_iter<K, PD, EDGE, FINAL, STEADY, U0>(T, C, pf, gp, s, d, g, L, i, c0, c1, in_lo, in_hi, top_reflect,
                                            bot_reflect, coef);
    if constexpr (sizeof...(Us) > 0)
        ws_group<K, PD, EDGE, FINAL, STEADY, Us...>(T, C, pf, gp, s, d, g, L, i + 1, c0, c1, in_lo, in_hi,
                                                    top_reflect, bot_reflect, coef);
}

template <int K, int PD, bool EDGE, bool FINAL, int... Us>
__device__ __forceinline__ void ws_body(std::integer_sequence<int, Us...>, const double *__restrict__ s, double *d,
                                        const double *g, const WcLane &L, int c0, int c1, int in_lo, int in_hi,
                                        int top_reflect, int bot_reflect, double coef) {
    static_assert(PD % 3 == 0, "the base-row prefetch rotates with period 3");
    double2 T[K], C[K], pf[PD], gp[3];
#pragma unroll
    for (int q = 0; q < K; ++q) T[q] = C[q] = make_double2(0.0, 0.0);
    const int64_t ny = L.ny;
    const int i0 = c0 - K + 2, i1 = c1 + K;          // iterations [i0, i1)
    const int s_lo = c0 + K, s_hi = c1 + K - 1;      // every stage active for i in [s_lo, s_hi]
    {   // stage 0 folds rows i0-2 and i0-1 before the first iteration
        C[0] = wc_load(s, (int64_t)min(max(i0 - 2, in_lo), in_hi - 1) * ny, L);
        const double2 x = wc_load(s, (int64_t)min(max(i0 - 1, in_lo), in_hi - 1) * ny, L);
        double2 up = C[0];
        if (EDGE && i0 - 1 == top_reflect) up = x;
        double leftA = dpp_from_lane_below(x.y), rightB = dpp_from_lane_above(x.x);
        if (EDGE) {
            leftA = L.l0 ? x.x : leftA;
            rightB = L.rN ? x.y : rightB;
        }
        T[0] = make_double2((fma(-4.0, x.x, up.x + leftA)) + x.y, (fma(-4.0, x.y, up.y + x.x)) + rightB);
        C[0] = x;
    }
#pragma unroll
    for (int u = 0; u < PD; ++u) pf[u] = wc_load(s, (int64_t)min(max(i0 + u, in_lo), in_hi - 1) * ny, L);
#pragma unroll
    for (int u = 0; u < 3; ++u)
        gp[u] = FINAL ? wc_load(g, (int64_t)min(max(i0 - K + u, c0), c1 - 1) * ny, L) : make_double2(0.0, 0.0);
#define WS_ARGS T, C, pf, gp, s, d, g, L, i, c0, c1, in_lo, in_hi, top_reflect, bot_reflect, coef
    int i = i0;
    for (; i + PD <= i1 && i < s_lo; i += PD) ws_group<K, PD, EDGE, FINAL, false, Us...>(WS_ARGS);   // fill
    for (; i + PD - 1 <= s_hi; i += PD) ws_group<K, PD, EDGE, FINAL, true, Us...>(WS_ARGS);          // steady
    for (; i + PD <= i1; i += PD) ws_group<K, PD, EDGE, FINAL, false, Us...>(WS_ARGS);               // drain
    ((i + Us < i1 ? ws_iter<K, PD, EDGE, FINAL, false, Us>(T, C, pf, gp, s, d, g, L, i + Us, c0, c1, in_lo, in_hi,
                                                           top_reflect, bot_reflect, coef)
                  : void()),
     ...);
#undef WS_ARGS
}

template <int K, int PD, bool FINAL, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void k_diffuse_wls(VK_WL_PARAMS) {
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
        ws_body<K, PD, true, FINAL>(std::make_integer_sequence<int, PD>(), s, d, g, L, c0, c1, in_lo, in_hi,
                                    top_reflect, bot_reflect, coef);
    else
        ws_body<K, PD, false, FINAL>(std::make_integer_sequence<int, PD>(), s, d, g, L, c0, c1, in_lo, in_hi,
                                     top_reflect, bot_reflect, coef);
}

template <int K, int WPE>
void launch_wls(hipStream_t st, const double *src, double *dst, const double *f0, int nf, int64_t fs, int ny,
                int out_lo, int out_hi, int in_lo, int in_hi, int top, int bot, double coef, const double *mm) {
    constexpr int KH = K + (K & 1);
    constexpr int W = WT_COLS - 2 * KH;
    const int tiles_x = (ny + W - 1) / W;
    const int rch = chunk_rows(out_hi - out_lo, tiles_x, nf);
    const int chunks_y = (out_hi - out_lo + rch - 1) / rch;
    const int waves = tiles_x * chunks_y * nf;
    if (f0)
        hipLaunchKernelGGL((k_diffuse_wls<K, 3, true, WPE>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst, f0,
                           fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef, mm);
    else
        hipLaunchKernelGGL((k_diffuse_wls<K, 3, false, WPE>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst,
                           f0, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef, mm);
}

}  // namespace

// ny must be even (the launcher in vk_lattice.hip routes odd widths elsewhere)
void vk_launch_wls(VK_STENCIL_LAUNCH_ARGS) {
#define VK_WS(KC, WPE) \
    case KC: launch_wls<KC, WPE>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm); break
    switch (k) {
        VK_WS(3, 4); VK_WS(5, 4); VK_WS(7, 4); VK_WS(9, 3); VK_WS(11, 3);
        default: break;
    }
#undef VK_WS
}
