// Fused-pass stencil kernels (temporal blocking), shared by the stencil
// translation units.  Each vk_stencil_*.hip instantiates one family of
// launchers, so the (many) template instantiations compile in parallel;
// vk_lattice.hip (vk_diffuse) calls them through vk_stencil_launch.h.
#pragma once

#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <utility>

#include "vk_internal.h"
#include "vk_stencil_launch.h"

// ---------------------------------------------------------------------------
// Temporally blocked stencil: K substeps per pass over HBM.  A tile streams its
// input rows top to bottom once; substep q is a pipeline stage holding its rows
// in VGPRs, so a pass reads (chunk + 2K) rows and writes chunk rows instead of K
// reads and K writes.  The arithmetic per cell and substep is the reference's
// ((up + left) + (-4*c)) + right) + down, c + coef*lap -- fma(-4, c, s) is
// bit-identical to s + (-4*c) because -4*c is exact.
// ---------------------------------------------------------------------------

// ---------------------------------------------------------------------------
// Wave tiles: one wavefront = one independent tile of 128 columns (two
// adjacent columns per lane), so there is no LDS and no barrier at all.  The
// left/right neighbours come from the lane itself (A<->B) and from the
// adjacent lanes through DPP wave shifts (v_mov_b32_dpp wave_shr:1 /
// wave_shl:1); the tile's outer KH columns per side are the halo that the K
// fused substeps eat into.  Loads/stores are 16 B per lane.
// ---------------------------------------------------------------------------

constexpr int WT_COLS = 128;

// bound_ctrl = true: the lane shifted in from outside the wave reads 0 (that
// lane is tile halo), so no "old" operand has to be materialised.
__device__ __forceinline__ double dpp_from_lane_below(double v) {  // lane l <- lane l-1
    int2 x = __builtin_bit_cast(int2, v);
    int2 y;
    y.x = __builtin_amdgcn_mov_dpp(x.x, 0x138, 0xf, 0xf, true);
    y.y = __builtin_amdgcn_mov_dpp(x.y, 0x138, 0xf, 0xf, true);
    return __builtin_bit_cast(double, y);
}

__device__ __forceinline__ double dpp_from_lane_above(double v) {  // lane l <- lane l+1
    int2 x = __builtin_bit_cast(int2, v);
    int2 y;
    y.x = __builtin_amdgcn_mov_dpp(x.x, 0x130, 0xf, 0xf, true);
    y.y = __builtin_amdgcn_mov_dpp(x.y, 0x130, 0xf, 0xf, true);
    return __builtin_bit_cast(double, y);
}

// Full-tile store of one lane's two columns.  VK_WL_NT_STORE (set by a
// translation unit before including this header) makes it a streaming store:
// the written plane is read again only by the next pass.
__device__ __forceinline__ void wl_store(double *o, double2 v) {
#ifdef VK_WL_NT_STORE
    typedef double d2v __attribute__((ext_vector_type(2)));
    d2v w = {v.x, v.y};
    __builtin_nontemporal_store(w, reinterpret_cast<d2v *>(o));
#else
    *reinterpret_cast<double2 *>(o) = v;
#endif
}

struct WtLane {
    int cA;              // this lane's first column (cB = cA + 1)
    int ny;
    bool wA, wB;         // writes its column A / B
    bool lA, rA, lB, rB; // reflect flags (EDGE tiles only)
};

// Row x clamped into the pass's input rows [lo, hi).
__device__ __forceinline__ int64_t wl_row(const WtLane &L, int x, int lo, int hi) {
    (void)L;
    return (int64_t)min(max(x, lo), hi - 1);
}

template <bool EDGE>
__device__ __forceinline__ double2 wt_load(const double *__restrict__ p, int64_t row_off, const WtLane &L) {
    if (!EDGE) {
        return *reinterpret_cast<const double2 *>(p + row_off + L.cA);
    }
    const int a = min(max(L.cA, 0), L.ny - 1), b = min(max(L.cA + 1, 0), L.ny - 1);
    return make_double2(p[row_off + a], p[row_off + b]);
}

// ---------------------------------------------------------------------------
// Lag-1 pipeline (variants 2/3/4/6): stage q consumes stage q-1's output of the SAME iteration
// (stage q computes row i-1-q at iteration i).  At the start of an iteration
// each stage holds only two live rows (up, centre) instead of three, so the
// register footprint drops from ~3K to ~2K row-pairs and more waves fit per
// SIMD; the price is a dependency chain through the stages of one iteration,
// which the unrolled body and the extra waves overlap.  Slot roles rotate with
// the iteration phase U (period 3): up = S[U], centre = S[U+1], fresh = S[U+2].
// ---------------------------------------------------------------------------

// PD = rows prefetched ahead in VGPRs (a multiple of 3: the slot roles rotate with period 3)
template <int K, int PD, bool EDGE, bool FINAL, bool STEADY, int U>
__device__ __forceinline__ void wl_iter(double2 (&S0)[K], double2 (&S1)[K], double2 (&S2)[K], double2 (&pf)[PD], double2 (&gp)[3],
                                        const double *__restrict__ s, double *d,
                                        const double *g, const WtLane &L, int i, int c0, int c1,
                                        int in_lo, int in_hi, int top_reflect, int bot_reflect, double coef) {
    constexpr int R = U % 3;
    double2(&UP)[K] = R == 0 ? S0 : (R == 1 ? S1 : S2);
    double2(&CN)[K] = R == 0 ? S1 : (R == 1 ? S2 : S0);
    double2(&FR)[K] = R == 0 ? S2 : (R == 1 ? S0 : S1);
    const int64_t ny = L.ny;
    FR[0] = pf[U];                                                                      // row i
    pf[U] = wt_load<EDGE>(s, wl_row(L, i + PD, in_lo, in_hi) * ny, L);             // row i+PD
    const int r_out = i - K;
    const bool row_ok = STEADY || (r_out >= c0 && r_out < c1);
    double2 base = make_double2(0.0, 0.0);
    if (FINAL) {   // base row r_out arrived 3 iterations ago; fetch row r_out+3 (clamped into the chunk)
        base = gp[R];
        if (L.wA || L.wB) gp[R] = wt_load<EDGE>(g, (int64_t)min(max(r_out + 3, c0), c1 - 1) * ny, L);
    }
#pragma unroll
    for (int q = 0; q < K; ++q) {
        // stage q is useful for rows [c0-(K-1-q), c1+(K-1-q)), i.e. i in [c0-K+2+2q, c1+K)
        if (!STEADY && (i < c0 - K + 2 + 2 * q || i >= c1 + K)) continue;
        const int r = i - 1 - q;
        const double2 cen = CN[q];
        const double2 up = (EDGE && r == top_reflect) ? cen : UP[q];
        const double2 dn = (EDGE && r == bot_reflect) ? cen : FR[q];
        double leftA = dpp_from_lane_below(cen.y), rightB = dpp_from_lane_above(cen.x);
        double rightA = cen.y, leftB = cen.x;
        if (EDGE) {
            leftA = L.lA ? cen.x : leftA;
            rightA = L.rA ? cen.x : rightA;
            leftB = L.lB ? cen.y : leftB;
            rightB = L.rB ? cen.y : rightB;
        }
        const double lapA = ((fma(-4.0, cen.x, up.x + leftA)) + rightA) + dn.x;
        const double lapB = ((fma(-4.0, cen.y, up.y + leftB)) + rightB) + dn.y;
        double2 v = make_double2(cen.x + coef * lapA, cen.y + coef * lapB);
        if (q + 1 < K) {
            FR[q + 1] = v;
        } else if (row_ok) {
            if (FINAL) v = make_double2(base.x + (v.x - base.x), base.y + (v.y - base.y));
            double *o = d + (int64_t)r_out * ny + L.cA;
            if (!EDGE) {
                if (L.wA) wl_store(o, v);
            } else {
                if (L.wA) o[0] = v.x;
                if (L.wB) o[1] = v.y;
            }
        }
    }
}

template <int K, int PD, bool EDGE, bool FINAL, bool STEADY, int U0, int... Us>
__device__ __forceinline__ void wl_group(double2 (&S0)[K], double2 (&S1)[K], double2 (&S2)[K],
                                         double2 (&pf)[PD], double2 (&gp)[3], const double *__restrict__ s, double *d,
                                         const double *g, const WtLane &L, int i, int c0, int c1,
                                         int in_lo, int in_hi, int top_reflect, int bot_reflect, double coef) {
    wl_iter<K, PD, EDGE, FINAL, STEADY, U0>(S0, S1, S2, pf, gp, s, d, g, L, i, c0, c1, in_lo, in_hi,
                                                  top_reflect, bot_reflect, coef);
    if constexpr (sizeof...(Us) > 0)
        wl_group<K, PD, EDGE, FINAL, STEADY, Us...>(S0, S1, S2, pf, gp, s, d, g, L, i + 1, c0, c1, in_lo,
                                                          in_hi, top_reflect, bot_reflect, coef);
}

template <int K, int PD, bool EDGE, bool FINAL, int... Us>
__device__ __forceinline__ void diffuse_wl_loop(std::integer_sequence<int, Us...>, double2 (&S0)[K],
                                                double2 (&S1)[K], double2 (&S2)[K], double2 (&pf)[PD], double2 (&gp)[3],
                                                const double *__restrict__ s, double *d,
                                                const double *g, const WtLane &L, int c0, int c1,
                                                int in_lo, int in_hi, int top_reflect, int bot_reflect,
                                                double coef) {
    const int i0 = c0 - K + 2, i1 = c1 + K;          // iterations [i0, i1)
    const int s_lo = c0 + K, s_hi = c1 + K - 1;      // every stage active for i in [s_lo, s_hi]
#define WL_ARGS S0, S1, S2, pf, gp, s, d, g, L, i, c0, c1, in_lo, in_hi, top_reflect, bot_reflect, coef
    constexpr int NU = PD;                           // iterations per unrolled group
    int i = i0;
    for (; i + NU <= i1 && i < s_lo; i += NU) wl_group<K, PD, EDGE, FINAL, false, Us...>(WL_ARGS);   // fill
    for (; i + NU - 1 <= s_hi; i += NU) wl_group<K, PD, EDGE, FINAL, true, Us...>(WL_ARGS);          // steady
    for (; i + NU <= i1; i += NU) wl_group<K, PD, EDGE, FINAL, false, Us...>(WL_ARGS);               // drain
    // tail: fewer than NU iterations, phases 0.. in order
    ((i + Us < i1 ? wl_iter<K, PD, EDGE, FINAL, false, Us>(S0, S1, S2, pf, gp, s, d, g, L, i + Us, c0, c1,
                                                              in_lo, in_hi, top_reflect, bot_reflect, coef)
                  : void()), ...);
#undef WL_ARGS
}

template <int K, int PD, bool EDGE, bool FINAL>
__device__ __forceinline__ void diffuse_wl_body(const double *__restrict__ s, double *d,
                                                const double *g, const WtLane &L, int c0, int c1,
                                                int in_lo, int in_hi, int top_reflect, int bot_reflect,
                                                double coef) {
    double2 S0[K], S1[K], S2[K], pf[PD], gp[3];
#pragma unroll
    for (int q = 0; q < K; ++q) S0[q] = S1[q] = S2[q] = make_double2(0.0, 0.0);
    const int64_t ny = L.ny;
    const int i0 = c0 - K + 2;
    // stage 0's window before the first iteration: up = row i0-2, centre = row i0-1
    S0[0] = wt_load<EDGE>(s, wl_row(L, i0 - 2, in_lo, in_hi) * ny, L);
    S1[0] = wt_load<EDGE>(s, wl_row(L, i0 - 1, in_lo, in_hi) * ny, L);
#pragma unroll
    for (int u = 0; u < PD; ++u) pf[u] = wt_load<EDGE>(s, wl_row(L, i0 + u, in_lo, in_hi) * ny, L);
#pragma unroll
    for (int u = 0; u < 3; ++u)   // FINAL: base rows of the first 3 output rows (i0 - K + u)
        gp[u] = FINAL && (L.wA || L.wB)
                    ? wt_load<EDGE>(g, (int64_t)min(max(i0 - K + u, c0), c1 - 1) * ny, L)
                    : make_double2(0.0, 0.0);
    diffuse_wl_loop<K, PD, EDGE, FINAL>(std::make_integer_sequence<int, PD>(), S0, S1, S2, pf, gp, s, d, g, L,
                                              c0, c1, in_lo, in_hi, top_reflect, bot_reflect, coef);
}

// The stencil work of one wave: its tile of plane f, output rows [c0, c1)
template <int K, int PD, bool FINAL>
__device__ __forceinline__ void diffuse_wl_tile_body(const double *__restrict__ src, double *dst, const double *f0,
                                                     int64_t field_stride, int ny, int in_lo, int in_hi,
                                                     int top_reflect, int bot_reflect, double coef, int f, int x0,
                                                     int c0, int c1, int lane) {
    constexpr int KH = K + (K & 1);
    WtLane L;
    L.ny = ny;
    L.cA = x0 - KH + 2 * lane;
    const int cB = L.cA + 1;
    L.wA = lane >= KH / 2 && lane < 64 - KH / 2 && L.cA < ny;
    L.wB = lane >= KH / 2 && lane < 64 - KH / 2 && cB < ny;
    L.lA = L.cA == 0;
    L.rA = L.cA == ny - 1;
    L.lB = cB == 0;
    L.rB = cB == ny - 1;
    const double *s = src + (int64_t)f * field_stride;
    double *d = dst + (int64_t)f * field_stride;
    const double *g = f0 ? f0 + (int64_t)f * field_stride : nullptr;
    const bool edge = (x0 - KH <= 0) || (x0 - KH + WT_COLS >= ny) || (ny & 1) ||
                      (top_reflect >= c0 - 2 * K - 2 && top_reflect <= c1 + 2 * K) ||
                      (bot_reflect >= c0 - 2 * K - 2 && bot_reflect <= c1 + 2 * K);
    if (edge)
        diffuse_wl_body<K, PD, true, FINAL>(s, d, g, L, c0, c1, in_lo, in_hi, top_reflect, bot_reflect, coef);
    else
        diffuse_wl_body<K, PD, false, FINAL>(s, d, g, L, c0, c1, in_lo, in_hi, top_reflect, bot_reflect, coef);
}

// Dispatch order of a pass's tiles (wave index -> tile): the tiles that run the
// general edge body (the pair-sum pass: about 2.6x the interior body's instructions) first -- every
// column of the ea top and eb bottom chunk rows whose reflected row is in reach,
// then the two side columns of the other rows -- and the interior tiles after
// them, plane-major.  In plane-major order the last chunk rows of the last plane,
// all edge tiles, were the last waves of the pass and ran on alone: the C4 step
// took 1.517 ms against 1.360 with this order (profiles/r05/r05v/).
__device__ __forceinline__ void vk_tile_of(int wave, int tiles_x, int chunks_y, int nf, int ea, int eb, int &tx,
                                           int &ty, int &f) {
    const int re = ea + eb;
    if (re <= chunks_y) {
        const int mid = chunks_y - re, side = tiles_x < 2 ? tiles_x : 2, inner = tiles_x - side;
        const int na = nf * re * tiles_x, nb = nf * mid * side;
        if (wave < na) {
            const int per = re * tiles_x;
            f = wave / per;
            const int r = wave - f * per, j = r / tiles_x;
            tx = r - j * tiles_x;
            ty = j < ea ? j : chunks_y - eb + (j - ea);
            return;
        }
        if (wave < na + nb) {
            const int w = wave - na, per = mid * side;
            f = w / per;
            const int r = w - f * per;
            ty = ea + r / side;
            tx = (r % side) == 0 ? 0 : tiles_x - 1;
            return;
        }
        const int w = wave - na - nb, per = mid * inner;   // inner > 0 here: wave < all tiles
        f = w / per;
        const int r = w - f * per;
        ty = ea + r / inner;
        tx = 1 + r % inner;
        return;
    }
    tx = wave % tiles_x;
    ty = (wave / tiles_x) % chunks_y;
    f = wave / (tiles_x * chunks_y);
}

// XCD-aware block order (speed only: any bijection computes the same cells).
// Blocks are dealt round-robin over the 8 XCDs, so blocks b and b + 8 share an
// L2.  Within each window of 8 * M blocks, block b takes slot (b % 8) * M +
// (b / 8) % M of the window: each XCD runs M consecutive blocks of the order
// above, side-by-side tiles that share their halo columns through its L2.  The
// pair-sum pass uses M = 4 (16 tiles): C4 reads 371 -> 355 MB per launch; M = 9
// was slower, and the stage-split pass (one tile per block) gained nothing
// (profiles/r05/r05xcd*).
template <int M>
__device__ __forceinline__ int vk_xcd_block(int b, int nb) {
    if constexpr (M > 1) {
        constexpr int S = 8 * M;
        if (b < nb / S * S) {
            const int i = b % S;
            return b - i + (i & 7) * M + (i >> 3);
        }
    }
    return b;
}

// Edge chunk rows of a pass (host): the leading / trailing chunks whose reflected
// rows are in reach -- the kernel's `ey` rule -- for the edge-first order.
static inline void vk_edge_chunks(int K, int out_lo, int out_hi, int rch, int chunks_y, int top, int bot, int &ea,
                                  int &eb) {
    auto ey = [&](int ty) {
        const int c0 = out_lo + ty * rch, c1 = std::min(c0 + rch, out_hi);
        return (top >= c0 - 2 * K - 2 && top <= c1 + 2 * K) || (bot >= c0 - 2 * K - 2 && bot <= c1 + 2 * K);
    };
    ea = 0;
    while (ea < chunks_y && ey(ea)) ++ea;
    eb = 0;
    while (ea + eb < chunks_y && ey(chunks_y - 1 - eb)) ++eb;
}

template <int K, int PD, bool FINAL>
__device__ __forceinline__ void diffuse_wl_tile(const double *__restrict__ src, double *dst,
                                                const double *f0, int64_t field_stride, int ny,
                                                int out_lo, int out_hi, int in_lo, int in_hi, int top_reflect,
                                                int bot_reflect, int rows_per_chunk, int tiles_x, int chunks_y,
                                                int n_fields, double coef, const double *__restrict__ uniform,
                                                const VkPsCouple &cp, int ea, int eb) {
    constexpr int KH = K + (K & 1);
    constexpr int W = WT_COLS - 2 * KH;
    // (An XCD-contiguous tile order -- each XCD's L2 serving its tiles' shared
    // halo columns -- measured 4 % slower on 4096^2: the halo re-reads already
    // hit the die-level Infinity Cache, so plain round-robin order is kept.)
    const int wave = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
    const int lane = threadIdx.x & 63;
    if (wave >= tiles_x * chunks_y * n_fields) return;
    int tx, ty, f;
    vk_tile_of(wave, tiles_x, chunks_y, n_fields, ea, eb, tx, ty, f);   // edge tiles first
    const int c0 = out_lo + ty * rows_per_chunk;
    const int c1 = min(c0 + rows_per_chunk, out_hi);
    const int x0 = tx * W;
    // agent coupling (vk_diffuse_coupled): the gather reads the plane before this pass
    // changes anything; a uniform plane keeps its values and still takes the exchange
    if (cp.mode & 1) vk_couple_gather(cp, src + (int64_t)f * field_stride, f, ny, x0, W, c0, c1, lane);
    if (!(uniform && uniform[2 * f] == uniform[2 * f + 1]))
        diffuse_wl_tile_body<K, PD, FINAL>(src, dst, f0, field_stride, ny, in_lo, in_hi, top_reflect,
                                                 bot_reflect, coef, f, x0, c0, c1, lane);
    if (cp.mode & 2) vk_couple_exchange(cp, dst + (int64_t)f * field_stride, f, ny, x0, W, c0, c1, lane);
}

// Aliasing: the FINAL pass writes the field it also reads as the base plane
// (dst == f0, vk_diffuse), so only the source plane is __restrict__; each base
// load feeds the store of the same cell, later in program order.
#define VK_WL_PARAMS                                                                                           \
    const double *__restrict__ src, double *dst, const double *f0, int64_t field_stride, \
        int ny, int out_lo, int out_hi, int in_lo, int in_hi, int top_reflect, int bot_reflect, int rows_per_chunk, \
        int tiles_x, int chunks_y, int n_fields, double coef, const double *__restrict__ uniform, const VkPsCouple cp, \
        int ea, int eb
#define VK_WL_ARGS                                                                                             \
    src, dst, f0, field_stride, ny, out_lo, out_hi, in_lo, in_hi, top_reflect, bot_reflect, rows_per_chunk,      \
        tiles_x, chunks_y, n_fields, coef, uniform, cp, ea, eb

#ifndef VK_WL_WAVES_ATTR
#define VK_WL_WAVES_ATTR
#endif
template <int K, int PD, bool FINAL>
__global__ __launch_bounds__(256) VK_WL_WAVES_ATTR void k_diffuse_wl(VK_WL_PARAMS) {
    diffuse_wl_tile<K, PD, FINAL>(VK_WL_ARGS);
}

// Rows per wave tile: g_stencil_rows, or (auto) by the height of the rows the
// pass writes -- small row bands (multi-GPU strong scaling) trade pipeline
// fill for more waves.
static int chunk_rows(int out_rows, int tiles_x, int nf) {
    if (::g_stencil_rows > 0) return ::g_stencil_rows;
    // auto: the strong-scaling sweep of 4096^2 x 2 bands (scripts/halo_sweep.py,
    // profiles/r02_halo_sweep/) is fastest with 64-row tiles on the whole
    // plane, 32 on 1/2 and 1/4 bands, 16 on 1/8 bands.  Narrower lattices have
    // fewer tile columns: halve the rows until the pass has >= 1500 waves (a
    // 1024^2 x 2 pass with 64-row tiles is 320 waves on 1024 SIMDs and takes
    // 0.58 ms per 100 substeps; with 8-row tiles 0.35 ms, profiles/r02d_c3/)
    int rows = out_rows >= 3000 ? 64 : (out_rows >= 1000 ? 32 : 16);
    while (rows > 8 && (int64_t)tiles_x * ((out_rows + rows - 1) / rows) * nf < 1500) rows /= 2;
    return rows;
}
