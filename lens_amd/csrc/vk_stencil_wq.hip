// Four-column wave tile (variant 8): the lag-1 pipeline of k_diffuse_wl with
// each lane owning FOUR adjacent columns of a 256-column tile.  Three of a
// lane's four left/right neighbours are its own registers; only the outer two
// come through a DPP wave shift, so the VALU count per cell and substep drops
// from 6 FP64 + 2 DPP moves to 6 FP64 + 1, and the tile's halo (KH columns per
// side) is amortised over 256 - 2*KH output columns instead of 128 - 2*KH.
// Same arithmetic, same order, bit-identical to the other variants.
#define VK_WL_NT_STORE 1
#include "vk_stencil_kernels.h"

namespace {

constexpr int WQ_COLS = 256;

struct R4 {
    double x[4];
};

struct WqLane {
    int cA;        // first of this lane's four columns
    int ny;
    bool w[4];     // writes column cA + k
    bool l[4], r[4];
};

template <bool EDGE>
__device__ __forceinline__ R4 wq_load(const double *__restrict__ p, int64_t row_off, const WqLane &L) {
    R4 o;
    if (!EDGE) {
        const double2 a = *reinterpret_cast<const double2 *>(p + row_off + L.cA);
        const double2 b = *reinterpret_cast<const double2 *>(p + row_off + L.cA + 2);
        o.x[0] = a.x;
        o.x[1] = a.y;
        o.x[2] = b.x;
        o.x[3] = b.y;
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k) o.x[k] = p[row_off + min(max(L.cA + k, 0), L.ny - 1)];
    }
    return o;
}

template <bool EDGE>
__device__ __forceinline__ void wq_store(double *o, const R4 &v, const WqLane &L) {
    if (!EDGE) {   // pairs (0,1) and (2,3) are written or skipped together (even halo, even ny)
        if (L.w[0]) wl_store(o, make_double2(v.x[0], v.x[1]));
        if (L.w[2]) wl_store(o + 2, make_double2(v.x[2], v.x[3]));
    } else {
#pragma unroll
        for (int k = 0; k < 4; ++k)
            if (L.w[k]) o[k] = v.x[k];
    }
}

template <int K, int PD, bool EDGE, bool FINAL, bool STEADY, int U>
__device__ __forceinline__ void wq_iter(R4 (&S0)[K], R4 (&S1)[K], R4 (&S2)[K], R4 (&pf)[PD], R4 (&gp)[3],
                                        const double *__restrict__ s, double *d, const double *g, const WqLane &L,
                                        int i, int c0, int c1, int in_lo, int in_hi, int top_reflect,
                                        int bot_reflect, double coef) {
    constexpr int R = U % 3;
    R4(&UP)[K] = R == 0 ? S0 : (R == 1 ? S1 : S2);
    R4(&CN)[K] = R == 0 ? S1 : (R == 1 ? S2 : S0);
    R4(&FR)[K] = R == 0 ? S2 : (R == 1 ? S0 : S1);
    const int64_t ny = L.ny;
    const bool writer = L.w[0] || L.w[1] || L.w[2] || L.w[3];
    __builtin_amdgcn_sched_barrier(0);   // keep iterations apart: interleaving them only raises VGPR pressure
    FR[0] = pf[U];                                                                        // row i
    pf[U] = wq_load<EDGE>(s, (int64_t)min(max(i + PD, in_lo), in_hi - 1) * ny, L);     // row i+PD
    const int r_out = i - K;
    const bool row_ok = STEADY || (r_out >= c0 && r_out < c1);
    R4 base;
    if (FINAL) {   // base row r_out arrived 3 iterations ago; fetch row r_out+3 (clamped into the chunk)
        base = gp[R];
        if (writer) gp[R] = wq_load<EDGE>(g, (int64_t)min(max(r_out + 3, c0), c1 - 1) * ny, L);
    }
#pragma unroll
    for (int q = 0; q < K; ++q) {
        if (!STEADY && (i < c0 - K + 2 + 2 * q || i >= c1 + K)) {
            // an idle stage's output slot is dead: say so, or its stale value stays live
            if (q + 1 < K)
#pragma unroll
                for (int k = 0; k < 4; ++k) FR[q + 1].x[k] = __builtin_nondeterministic_value(0.0);
            continue;
        }
        const int r = i - 1 - q;
        const R4 cen = CN[q];
        const R4 up = (EDGE && r == top_reflect) ? cen : UP[q];
        const R4 dn = (EDGE && r == bot_reflect) ? cen : FR[q];
        double lf[4], rt[4];
        lf[0] = dpp_from_lane_below(cen.x[3]);
        rt[3] = dpp_from_lane_above(cen.x[0]);
#pragma unroll
        for (int k = 1; k < 4; ++k) lf[k] = cen.x[k - 1];
#pragma unroll
        for (int k = 0; k < 3; ++k) rt[k] = cen.x[k + 1];
        if (EDGE) {
#pragma unroll
            for (int k = 0; k < 4; ++k) {
                lf[k] = L.l[k] ? cen.x[k] : lf[k];
                rt[k] = L.r[k] ? cen.x[k] : rt[k];
            }
        }
        R4 v;
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const double lap = ((fma(-4.0, cen.x[k], up.x[k] + lf[k])) + rt[k]) + dn.x[k];
            v.x[k] = cen.x[k] + coef * lap;
        }
        if (q + 1 < K) {
            FR[q + 1] = v;
        } else if (row_ok) {
            if (FINAL) {
#pragma unroll
                for (int k = 0; k < 4; ++k) v.x[k] = base.x[k] + (v.x[k] - base.x[k]);
            }
            wq_store<EDGE>(d + (int64_t)r_out * ny + L.cA, v, L);
        }
    }
}

template <int K, int PD, bool EDGE, bool FINAL, bool STEADY, int U0, int... Us>
__device__ __forceinline__ void wq_group(R4 (&S0)[K], R4 (&S1)[K], R4 (&S2)[K], R4 (&pf)[PD], R4 (&gp)[3],
                                         const double *__restrict__ s, double *d, const double *g, const WqLane &L,
                                         int i, int c0, int c1, int in_lo, int in_hi, int top_reflect,
                                         int bot_reflect, double coef) {
    wq_iter<K, PD, EDGE, FINAL, STEADY, U0>(S0, S1, S2, pf, gp, s, d, g, L, i, c0, c1, in_lo, in_hi, top_reflect,
                                            bot_reflect, coef);
    if constexpr (sizeof...(Us) > 0)
        wq_group<K, PD, EDGE, FINAL, STEADY, Us...>(S0, S1, S2, pf, gp, s, d, g, L, i + 1, c0, c1, in_lo, in_hi,
                                                    top_reflect, bot_reflect, coef);
}

template <int K, int PD, bool EDGE, bool FINAL, int... Us>
__device__ __forceinline__ void wq_body(std::integer_sequence<int, Us...>, const double *__restrict__ s, double *d,
                                        const double *g, const WqLane &L, int c0, int c1, int in_lo, int in_hi,
                                        int top_reflect, int bot_reflect, double coef) {
    R4 S0[K], S1[K], S2[K], pf[PD], gp[3];
#pragma unroll
    for (int q = 0; q < K; ++q)
#pragma unroll
        for (int k = 0; k < 4; ++k) S0[q].x[k] = S1[q].x[k] = S2[q].x[k] = 0.0;
    const int64_t ny = L.ny;
    const int i0 = c0 - K + 2, i1 = c1 + K;          // iterations [i0, i1)
    const int s_lo = c0 + K, s_hi = c1 + K - 1;      // every stage active for i in [s_lo, s_hi]
    S0[0] = wq_load<EDGE>(s, (int64_t)min(max(i0 - 2, in_lo), in_hi - 1) * ny, L);
    S1[0] = wq_load<EDGE>(s, (int64_t)min(max(i0 - 1, in_lo), in_hi - 1) * ny, L);
#pragma unroll
    for (int u = 0; u < PD; ++u) pf[u] = wq_load<EDGE>(s, (int64_t)min(max(i0 + u, in_lo), in_hi - 1) * ny, L);
    const bool writer = L.w[0] || L.w[1] || L.w[2] || L.w[3];
#pragma unroll
    for (int u = 0; u < 3; ++u) {
        if (FINAL && writer) {
            gp[u] = wq_load<EDGE>(g, (int64_t)min(max(i0 - K + u, c0), c1 - 1) * ny, L);
        } else {
#pragma unroll
            for (int k = 0; k < 4; ++k) gp[u].x[k] = 0.0;
        }
    }
#define WQ_ARGS S0, S1, S2, pf, gp, s, d, g, L, i, c0, c1, in_lo, in_hi, top_reflect, bot_reflect, coef
    int i = i0;
    for (; i + PD <= i1 && i < s_lo; i += PD) wq_group<K, PD, EDGE, FINAL, false, Us...>(WQ_ARGS);   // fill
    for (; i + PD - 1 <= s_hi; i += PD) wq_group<K, PD, EDGE, FINAL, true, Us...>(WQ_ARGS);          // steady
    for (; i + PD <= i1; i += PD) wq_group<K, PD, EDGE, FINAL, false, Us...>(WQ_ARGS);               // drain
    ((i + Us < i1 ? wq_iter<K, PD, EDGE, FINAL, false, Us>(S0, S1, S2, pf, gp, s, d, g, L, i + Us, c0, c1, in_lo,
                                                           in_hi, top_reflect, bot_reflect, coef)
                  : void()),
     ...);
#undef WQ_ARGS
}

template <int K, int PD, bool FINAL, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void k_diffuse_wq(VK_WL_PARAMS) {
    constexpr int KH = K + (K & 1);            // even halo: 16-B aligned pairs
    constexpr int W = WQ_COLS - 2 * KH;        // output columns per tile
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
    WqLane L;
    L.ny = ny;
    L.cA = x0 - KH + 4 * lane;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int c = L.cA + k;
        L.w[k] = c >= x0 && c < x0 + W && c < ny;
        L.l[k] = c == 0;
        L.r[k] = c == ny - 1;
    }
    const double *s = src + (int64_t)f * field_stride;
    double *d = dst + (int64_t)f * field_stride;
    const double *g = f0 ? f0 + (int64_t)f * field_stride : nullptr;
    const bool edge = (x0 - KH <= 0) || (x0 - KH + WQ_COLS >= ny) || (ny & 1) ||
                      (top_reflect >= c0 - 2 * K - 2 && top_reflect <= c1 + 2 * K) ||
                      (bot_reflect >= c0 - 2 * K - 2 && bot_reflect <= c1 + 2 * K);
    if (edge)
        wq_body<K, PD, true, FINAL>(std::make_integer_sequence<int, PD>(), s, d, g, L, c0, c1, in_lo, in_hi,
                                    top_reflect, bot_reflect, coef);
    else
        wq_body<K, PD, false, FINAL>(std::make_integer_sequence<int, PD>(), s, d, g, L, c0, c1, in_lo, in_hi,
                                     top_reflect, bot_reflect, coef);
}

template <int K, int PD, int WPE>
void launch_wq(hipStream_t st, const double *src, double *dst, const double *f0, int nf, int64_t fs, int ny,
               int out_lo, int out_hi, int in_lo, int in_hi, int top, int bot, double coef, const double *mm) {
    constexpr int KH = K + (K & 1);
    constexpr int W = WQ_COLS - 2 * KH;
    const int tiles_x = (ny + W - 1) / W;
    const int rch = chunk_rows(out_hi - out_lo, tiles_x, nf);
    const int chunks_y = (out_hi - out_lo + rch - 1) / rch;
    const int waves = tiles_x * chunks_y * nf;
    if (f0)
        hipLaunchKernelGGL((k_diffuse_wq<K, 3, true, WPE>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst, f0, fs,
                           ny, out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef, mm);
    else
        hipLaunchKernelGGL((k_diffuse_wq<K, PD, false, WPE>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst, f0,
                           fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef, mm);
}

}  // namespace

void vk_launch_wq(VK_STENCIL_LAUNCH_ARGS) {
    switch (k) {
        case 3: launch_wq<3, 3, 3>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm); break;
        case 5: launch_wq<5, 3, 3>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm); break;
        case 7: launch_wq<7, 3, 2>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm); break;
        case 9: launch_wq<9, 3, 2>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm); break;
        case 11: launch_wq<11, 3, 2>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm); break;
        default: break;
    }
}
