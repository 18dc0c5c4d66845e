// Lag-1 wave tile, split stages with LDS-crossbar neighbours (variant 11).
//
// Variant 10 splits each stage into its in-iteration chain (lap = T + down,
// v = c + coef*lap) and the update of T for the next row, which needs the
// left/right neighbours of the stage's new centre row.  Those came from DPP
// moves: 4 of the 16 VALU instructions per lane and stage.  Here they come from
// ds_bpermute_b32 (the LDS crossbar: no LDS storage, no VALU issue slot), issued
// as soon as the new centre row exists and consumed D stages later, so the
// crossbar latency overlaps the chain: 12 VALU per lane and stage.
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

__device__ __forceinline__ double bperm(int addr, double v) {
    const int2 x = __builtin_bit_cast(int2, v);
    int2 y;
    y.x = __builtin_amdgcn_ds_bpermute(addr, x.x);
    y.y = __builtin_amdgcn_ds_bpermute(addr, x.y);
    return __builtin_bit_cast(double, y);
}

// a stage's update in flight: its old centre (the next row's "up") and the
// neighbours of its new centre, which is C[q] by then
struct Pend {
    double2 up;
    double left, right;
};

template <int K, bool EDGE>
__device__ __forceinline__ void wb_finish(double2 (&T)[K], const double2 (&C)[K], const Pend &p, int q, int rn,
                                          int top_reflect, const WcLane &L) {
    const double2 x = C[q];
    double2 up = p.up;
    if (EDGE && rn == top_reflect) up = x;
    double leftA = p.left, rightB = p.right;
    if (EDGE) {
        leftA = L.l0 ? x.x : leftA;
        rightB = L.rN ? x.y : rightB;
    }
    T[q] = make_double2((fma(-4.0, x.x, up.x + leftA)) + x.y, (fma(-4.0, x.y, up.y + x.x)) + rightB);
    asm volatile("" : "+v"(T[q].x), "+v"(T[q].y));   // here, not sunk to the end of the iteration
}

template <int K, int PD, int D, bool EDGE, bool FINAL, bool STEADY, int U>
__device__ __forceinline__ void wb_iter(double2 (&T)[K], double2 (&C)[K], double2 (&pf)[PD], double2 (&gp)[3],
                                        const double *__restrict__ s, double *d, const double *g, const WcLane &L,
                                        int ab, int aa, int i, int c0, int c1, int in_lo, int in_hi,
                                        int top_reflect, int bot_reflect, double coef) {
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
    Pend pend[K];
#pragma unroll
    for (int q = 0; q < K; ++q) {
        const bool cmp = STEADY || (i >= c0 - K + 2 + 2 * q && i < c1 + K);
        const bool upd = STEADY || (i >= c0 - K + 2 * q && i < c1 + K);
        if (upd) {   // neighbours of the new centre row i-q, through the LDS crossbar
            pend[q].left = bperm(ab, x.y);
            pend[q].right = bperm(aa, x.x);
        }
        double2 v;
        if (cmp) {
            double2 dn = x;
            if (EDGE && i - 1 - q == bot_reflect) dn = C[q];
            v = make_double2(C[q].x + coef * (T[q].x + dn.x), C[q].y + coef * (T[q].y + dn.y));
        }
        if (upd) {
            pend[q].up = C[q];
            C[q] = x;
        }
        if (q >= D) {
            const int p = q - D;
            if (STEADY || (i >= c0 - K + 2 * p && i < c1 + K))
                wb_finish<K, EDGE>(T, C, pend[p], p, i - p, top_reflect, L);
        }
        if (q + 1 < K) {
            x = v;
        } else if (row_ok) {
            if (FINAL) v = make_double2(base.x + (v.x - base.x), base.y + (v.y - base.y));
            if (L.w) wl_store(d + (int64_t)r_out * ny + L.cA, v);
        }
    }
#pragma unroll
    for (int p = (K > D ? K - D : 0); p < K; ++p)
        if (STEADY || (i >= c0 - K + 2 * p && i < c1 + K)) wb_finish<K, EDGE>(T, C, pend[p], p, i - p, top_reflect, L);
}

template <int K, int PD, int D, bool EDGE, bool FINAL, bool STEADY, int U0, int... Us>
__device__ __forceinline__ void wb_group(double2 (&T)[K], double2 (&C)[K], double2 (&pf)[PD], double2 (&gp)[3],
                                         const double *__restrict__ s, double *d, const double *g, const WcLane &L,
                                         int ab, int aa, int i, int c0, int c1, int in_lo, int in_hi,
                                         int top_reflect, int bot_reflect, double coef) {
    wb_iter<K, PD, D, EDGE, FINAL, STEADY, U0>(T, C, pf, gp, s, d, g, L, ab, aa, i, c0, c1, in_lo, in_hi,
                                               top_reflect, bot_reflect, coef);
    if constexpr (sizeof...(Us) > 0)
        wb_group<K, PD, D, EDGE, FINAL, STEADY, Us...>(T, C, pf, gp, s, d, g, L, ab, aa, i + 1, c0, c1, in_lo,
                                                       in_hi, top_reflect, bot_reflect, coef);
}

template <int K, int PD, bool EDGE, bool FINAL, int... Us>
__device__ __forceinline__ void wb_body(std::integer_sequence<int, Us...>, const double *__restrict__ s, double *d,
                                        const double *g, const WcLane &L, int c0, int c1, int in_lo, int in_hi,
                                        int top_reflect, int bot_reflect, double coef) {
    static_assert(PD % 3 == 0, "the base-row prefetch rotates with period 3");
    constexpr int D = 2;
    const int lane = threadIdx.x & 63;
    const int ab = ((lane + 63) & 63) << 2, aa = ((lane + 1) & 63) << 2;   // byte addresses of lanes l-1, l+1
    double2 T[K], C[K], pf[PD], gp[3];
#pragma unroll
    for (int q = 0; q < K; ++q) T[q] = C[q] = make_double2(0.0, 0.0);
    const int64_t ny = L.ny;
    const int i0 = c0 - K + 2, i1 = c1 + K;          // iterations [i0, i1)
    const int s_lo = c0 + K, s_hi = c1 + K - 1;      // every stage active for i in [s_lo, s_hi]
    {   // stage 0 folds rows i0-2 and i0-1 before the first iteration
        Pend p;
        p.up = wc_load(s, (int64_t)min(max(i0 - 2, in_lo), in_hi - 1) * ny, L);
        C[0] = wc_load(s, (int64_t)min(max(i0 - 1, in_lo), in_hi - 1) * ny, L);
        p.left = bperm(ab, C[0].y);
        p.right = bperm(aa, C[0].x);
        wb_finish<K, EDGE>(T, C, p, 0, i0 - 1, top_reflect, L);
    }
#pragma unroll
    for (int u = 0; u < PD; ++u) pf[u] = wc_load(s, (int64_t)min(max(i0 + u, in_lo), in_hi - 1) * ny, L);
#pragma unroll
    for (int u = 0; u < 3; ++u)
        gp[u] = FINAL ? wc_load(g, (int64_t)min(max(i0 - K + u, c0), c1 - 1) * ny, L) : make_double2(0.0, 0.0);
#define WB_ARGS T, C, pf, gp, s, d, g, L, ab, aa, i, c0, c1, in_lo, in_hi, top_reflect, bot_reflect, coef
    int i = i0;
    for (; i + PD <= i1 && i < s_lo; i += PD) wb_group<K, PD, D, EDGE, FINAL, false, Us...>(WB_ARGS);   // fill
    for (; i + PD - 1 <= s_hi; i += PD) wb_group<K, PD, D, EDGE, FINAL, true, Us...>(WB_ARGS);          // steady
    for (; i + PD <= i1; i += PD) wb_group<K, PD, D, EDGE, FINAL, false, Us...>(WB_ARGS);               // drain
    ((i + Us < i1 ? wb_iter<K, PD, D, EDGE, FINAL, false, Us>(T, C, pf, gp, s, d, g, L, ab, aa, i + Us, c0, c1,
                                                              in_lo, in_hi, top_reflect, bot_reflect, coef)
                  : void()),
     ...);
#undef WB_ARGS
}

template <int K, int PD, bool FINAL, int WPE>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(WPE, WPE))) void k_diffuse_wlb(VK_WL_PARAMS) {
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
        wb_body<K, PD, true, FINAL>(std::make_integer_sequence<int, PD>(), s, d, g, L, c0, c1, in_lo, in_hi,
                                    top_reflect, bot_reflect, coef);
    else
        wb_body<K, PD, false, FINAL>(std::make_integer_sequence<int, PD>(), s, d, g, L, c0, c1, in_lo, in_hi,
                                     top_reflect, bot_reflect, coef);
}

template <int K, int WPE>
void launch_wlb(hipStream_t st, const double *src, double *dst, const double *f0, int nf, int64_t fs, int ny,
                int out_lo, int out_hi, int in_lo, int in_hi, int top, int bot, double coef, const double *mm) {
    constexpr int KH = K + (K & 1);
    constexpr int W = WT_COLS - 2 * KH;
    const int tiles_x = (ny + W - 1) / W;
    const int rch = chunk_rows(out_hi - out_lo, tiles_x, nf);
    const int chunks_y = (out_hi - out_lo + rch - 1) / rch;
    const int waves = tiles_x * chunks_y * nf;
    if (f0)
        hipLaunchKernelGGL((k_diffuse_wlb<K, 3, true, (WPE < 3 ? WPE : 3)>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst, f0,
                           fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef, mm);
    else
        hipLaunchKernelGGL((k_diffuse_wlb<K, 3, false, WPE>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst,
                           f0, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef, mm);
}

}  // namespace

// ny must be even (the launcher in vk_lattice.hip routes odd widths elsewhere)
void vk_launch_wlb(VK_STENCIL_LAUNCH_ARGS) {
#define VK_WB(KC, WPE) \
    case KC: launch_wlb<KC, WPE>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm); break
    switch (k) {
        VK_WB(3, 4); VK_WB(5, 4); VK_WB(7, 4); VK_WB(9, 4); VK_WB(11, 3);
        default: break;
    }
#undef VK_WB
}
