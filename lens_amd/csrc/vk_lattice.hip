// diffusion_field lattice on MI355X (gfx950): 5-point reflect stencil,
// uniform-field detection, local-environment gather, agent exchange scatter.
//
// Reference semantics: vivarium/processes/diffusion_field.py:385-407
// (fixed 0.01 s substeps of f += (D/(dx*dy)*dt) * convolve(f, LAP,
// mode='reflect'), uniform skip, delta accumulated), :362-379 (local
// environments), vivarium/core/registry.py:149-183 (exchange updater),
// vivarium/library/lattice_utils.py:18-58 (bin sites / bin volume).
// Compiled with -ffp-contract=off: the Laplacian is summed up, left,
// -4*centre, right, down exactly as scipy.ndimage.convolve does, and the
// update is c + coef*lap with two roundings, so fields are bit-identical to
// the reference's.
//
// HBM layout: one plane per molecule, row-major [rows][ny] (axis 0 = x as in
// the reference's ndarray), planes field_stride apart.  A rank's plane holds
// its owned row band plus halo rows.

#include <math.h>
#include <stdint.h>

#include <algorithm>
#include <utility>


#include "vk_internal.h"

constexpr int ST_BX = 256;  // columns per block (4 waves, 2 KiB per row load)
constexpr int ST_RB = 16;   // rows walked per block

// One substep over rows [lo, hi) of every plane.  Each lane walks down a
// column keeping up/centre/down in registers: one new row load, two shifted
// loads (left/right: L1 hits on the lines the wave just fetched), one store.
__global__ __launch_bounds__(ST_BX) void k_diffuse_substep(const double *__restrict__ src,
                                                           double *__restrict__ dst,
                                                           const double *__restrict__ f0,
                                                           int64_t field_stride, int ny, int lo, int hi,
                                                           int top_reflect, int bot_reflect, double coef,
                                                           const double *__restrict__ uniform) {
    const int f = blockIdx.z;
    if (uniform && uniform[2 * f] == uniform[2 * f + 1]) return;  // uniform: delta is zero
    const int j = blockIdx.x * ST_BX + threadIdx.x;
    const int r0 = lo + blockIdx.y * ST_RB;
    if (j >= ny || r0 >= hi) return;
    const int r1 = min(r0 + ST_RB, hi);
    const double *s = src + (int64_t)f * field_stride;
    double *d = dst + (int64_t)f * field_stride;
    const double *g = f0 ? f0 + (int64_t)f * field_stride : nullptr;
    const int jl = j > 0 ? j - 1 : 0;
    const int jr = j < ny - 1 ? j + 1 : ny - 1;
    const int ru = (r0 == top_reflect) ? r0 : r0 - 1;
    double up = s[(int64_t)ru * ny + j];
    double c = s[(int64_t)r0 * ny + j];
    for (int r = r0; r < r1; ++r) {
        const int rd = (r == bot_reflect) ? r : r + 1;
        const double down = s[(int64_t)rd * ny + j];
        const double left = s[(int64_t)r * ny + jl];
        const double right = s[(int64_t)r * ny + jr];
        const double lap = (((up + left) + (-4.0 * c)) + right) + down;
        double v = c + coef * lap;
        if (g) {
            const double base = g[(int64_t)r * ny + j];
            v = base + (v - base);
        }
        d[(int64_t)r * ny + j] = v;
        up = c;
        c = down;
    }
}

// ---------------------------------------------------------------------------
// Temporally blocked stencil: K substeps per pass over HBM.
//
// A workgroup owns a tile of TB_BX columns (TB_BX-2K output columns + K halo
// columns per side) and a chunk of output rows; it streams its input rows
// top to bottom once.  Substep s (0-based) is a pipeline stage holding a
// three-row window (up, centre, newest) per column in VGPRs; at iteration i
// stage s produces row i-2s-1, and its output becomes stage s+1's newest
// row in iteration i+1, so all K stages of an iteration are independent and
// share ONE LDS exchange of centre values (left/right neighbours) and ONE
// barrier (LDS double-buffered by iteration parity).  HBM traffic per pass:
// one read of (chunk+2K) rows and one write of chunk rows, instead of K reads
// and K writes.  The arithmetic per cell and substep is the reference's
// ((up + left) + (-4*c)) + right) + down, c + coef*lap -- fma(-4, c, s) is
// bit-identical to s + (-4*c) because -4*c is exact.
// ---------------------------------------------------------------------------

constexpr int TB_BX = 256;

// One pipeline iteration with static register roles U (loop unrolled by 3, so
// the three-row windows rotate by renaming instead of v_mov).  For stage q:
// up = X[U], centre = X[U+1], newest = X[U+2] (mod 3); stage q-1's output is
// stage q's newest next iteration and lands in X[U] once stage q consumed it.
template <int K, bool EDGE, int U>
__device__ __forceinline__ void tb_iter(double (&xch)[2][K][TB_BX], double (&X0)[K], double (&X1)[K],
                                        double (&X2)[K], double (&pf)[3], const double *__restrict__ s,
                                        double *__restrict__ d, const double *__restrict__ g, int ny, int i,
                                        int c0, int c1, int in_lo, int in_hi, int top_reflect, int bot_reflect,
                                        int c, int cc, bool writer, int tl, int tr, bool left_edge,
                                        bool right_edge, double coef) {
    double(&UP)[K] = U == 0 ? X0 : (U == 1 ? X1 : X2);
    double(&CN)[K] = U == 0 ? X1 : (U == 1 ? X2 : X0);
    double(&NW)[K] = U == 0 ? X2 : (U == 1 ? X0 : X1);
    const int tid = threadIdx.x;
    NW[0] = pf[U];                                                    // row i, loaded 3 iterations ago
    pf[U] = s[(int64_t)min(max(i + 3, in_lo), in_hi - 1) * ny + cc];  // prefetch row i+3
    const int r_out = i - 2 * K + 1;
    const bool do_write = writer && r_out >= c0 && r_out < c1;
    double base = 0.0;
    if (g && do_write) base = g[(int64_t)r_out * ny + c];
    const int p = i & 1;
#pragma unroll
    for (int q = 0; q < K; ++q) xch[p][q][tid] = CN[q];
    __syncthreads();
#pragma unroll
    for (int q = K - 1; q >= 0; --q) {
        const int r = i - 2 * q - 1;
        const double cen = CN[q];
        const double up = (EDGE && r == top_reflect) ? cen : UP[q];
        const double dn = (EDGE && r == bot_reflect) ? cen : NW[q];
        const double lv = xch[p][q][tl], rv = xch[p][q][tr];
        const double lf = left_edge ? cen : lv;
        const double rt = right_edge ? cen : rv;
        const double lap = ((fma(-4.0, cen, up + lf)) + rt) + dn;
        const double v = cen + coef * lap;
        if (q + 1 < K) {
            UP[q + 1] = v;
        } else if (do_write) {
            d[(int64_t)r_out * ny + c] = g ? base + (v - base) : v;
        }
    }
}

// EDGE = the tile touches a reflecting boundary (global edge rows/columns);
// interior tiles (the vast majority) carry no boundary selects at all.
template <int K, bool EDGE>
__device__ __forceinline__ void diffuse_tb_body(double (&xch)[2][K][TB_BX], const double *__restrict__ s,
                                                double *__restrict__ d, const double *__restrict__ g, int ny,
                                                int c0, int c1, int in_lo, int in_hi, int top_reflect,
                                                int bot_reflect, int x0, double coef) {
    const int tid = threadIdx.x;
    const int c = x0 - K + tid;
    const int cc = min(max(c, 0), ny - 1);
    const bool left_edge = EDGE && (c == 0), right_edge = EDGE && (c == ny - 1);
    const bool writer = tid >= K && tid < TB_BX - K && c < ny;
    const int tl = max(tid - 1, 0), tr = min(tid + 1, TB_BX - 1);

    double X0[K], X1[K], X2[K], pf[3];
#pragma unroll
    for (int q = 0; q < K; ++q) X0[q] = X1[q] = X2[q] = 0.0;
    const int i0 = c0 - K, i1 = c1 + 2 * K - 1;
#pragma unroll
    for (int u = 0; u < 3; ++u) pf[u] = s[(int64_t)min(max(i0 + u, in_lo), in_hi - 1) * ny + cc];
#define TB_ARGS xch, X0, X1, X2, pf, s, d, g, ny
#define TB_REST c0, c1, in_lo, in_hi, top_reflect, bot_reflect, c, cc, writer, tl, tr, left_edge, right_edge, coef
    int i = i0;
    for (; i + 3 <= i1; i += 3) {
        tb_iter<K, EDGE, 0>(TB_ARGS, i, TB_REST);
        tb_iter<K, EDGE, 1>(TB_ARGS, i + 1, TB_REST);
        tb_iter<K, EDGE, 2>(TB_ARGS, i + 2, TB_REST);
    }
    if (i < i1) tb_iter<K, EDGE, 0>(TB_ARGS, i, TB_REST);
    if (i + 1 < i1) tb_iter<K, EDGE, 1>(TB_ARGS, i + 1, TB_REST);
#undef TB_ARGS
#undef TB_REST
}

template <int K>
__global__ __launch_bounds__(TB_BX) void k_diffuse_tb(const double *__restrict__ src, double *__restrict__ dst,
                                                      const double *__restrict__ f0, int64_t field_stride, int ny,
                                                      int out_lo, int out_hi, int in_lo, int in_hi,
                                                      int top_reflect, int bot_reflect, int rows_per_chunk,
                                                      double coef, const double *__restrict__ uniform) {
    const int f = blockIdx.z;
    if (uniform && uniform[2 * f] == uniform[2 * f + 1]) return;  // uniform plane: zero delta
    const int c0 = out_lo + blockIdx.y * rows_per_chunk;
    if (c0 >= out_hi) return;
    const int c1 = min(c0 + rows_per_chunk, out_hi);
    const int x0 = blockIdx.x * (TB_BX - 2 * K);
    __shared__ double xch[2][K][TB_BX];
    const double *s = src + (int64_t)f * field_stride;
    double *d = dst + (int64_t)f * field_stride;
    const double *g = f0 ? f0 + (int64_t)f * field_stride : nullptr;
    // rows this block touches: [c0-K-1, c1+2K); columns [x0-K-1, x0-K+TB_BX]
    const bool edge = (x0 - K - 1 <= 0) || (x0 - K + TB_BX >= ny - 1) ||
                      (top_reflect >= c0 - 3 * K - 2 && top_reflect <= c1 + 2 * K) ||
                      (bot_reflect >= c0 - 3 * K - 2 && bot_reflect <= c1 + 2 * K);
    if (edge)
        diffuse_tb_body<K, true>(xch, s, d, g, ny, c0, c1, in_lo, in_hi, top_reflect, bot_reflect, x0, coef);
    else
        diffuse_tb_body<K, false>(xch, s, d, g, ny, c0, c1, in_lo, in_hi, top_reflect, bot_reflect, x0, coef);
}

// ---------------------------------------------------------------------------
// Wave-tile variant: one wavefront = one independent tile of 128 columns (two
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

struct WtLane {
    int cA;              // this lane's first column (cB = cA + 1)
    int ny;
    bool wA, wB;         // writes its column A / B
    bool lA, rA, lB, rB; // reflect flags (EDGE tiles only)
};

template <bool EDGE>
__device__ __forceinline__ double2 wt_load(const double *__restrict__ p, int64_t row_off, const WtLane &L) {
    if (!EDGE) return *reinterpret_cast<const double2 *>(p + row_off + L.cA);
    const int a = min(max(L.cA, 0), L.ny - 1), b = min(max(L.cA + 1, 0), L.ny - 1);
    return make_double2(p[row_off + a], p[row_off + b]);
}

// STEADY: every stage is inside its useful row range (no fill/drain test),
// so the K stages are straight-line code the scheduler can interleave.
template <int K, bool EDGE, bool FINAL, bool STEADY, int U>
__device__ __forceinline__ void wt_iter(double2 (&X0)[K], double2 (&X1)[K], double2 (&X2)[K], double2 (&pf)[3],
                                        const double *__restrict__ s, double *__restrict__ d,
                                        const double *__restrict__ g, const WtLane &L, int i, int c0, int c1,
                                        int in_lo, int in_hi, int top_reflect, int bot_reflect, double coef) {
    double2(&UP)[K] = U == 0 ? X0 : (U == 1 ? X1 : X2);
    double2(&CN)[K] = U == 0 ? X1 : (U == 1 ? X2 : X0);
    double2(&NW)[K] = U == 0 ? X2 : (U == 1 ? X0 : X1);
    const int64_t ny = L.ny;
    NW[0] = pf[U];                                                                   // row i
    pf[U] = wt_load<EDGE>(s, (int64_t)min(max(i + 3, in_lo), in_hi - 1) * ny, L);  // prefetch row i+3
    const int r_out = i - 2 * K + 1;
    const bool row_ok = STEADY || (r_out >= c0 && r_out < c1);
    double2 base = make_double2(0.0, 0.0);
    if (FINAL && row_ok && (L.wA || L.wB)) base = wt_load<EDGE>(g, (int64_t)r_out * ny, L);
#pragma unroll
    for (int q = K - 1; q >= 0; --q) {
        // stage q only matters for output rows [c0-(K-1-q), c1+(K-1-q)):
        // skip the pipeline fill/drain iterations (wave-uniform branch)
        if (!STEADY && (i < c0 - K + 3 * q + 2 || i > c1 + K - 1 + q)) continue;
        const int r = i - 2 * q - 1;
        const double2 cen = CN[q];
        const double2 up = (EDGE && r == top_reflect) ? cen : UP[q];
        const double2 dn = (EDGE && r == bot_reflect) ? cen : NW[q];
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
            UP[q + 1] = v;
        } else if (row_ok) {
            if (FINAL) v = make_double2(base.x + (v.x - base.x), base.y + (v.y - base.y));
            double *o = d + (int64_t)r_out * ny + L.cA;
            if (!EDGE) {
                if (L.wA) *reinterpret_cast<double2 *>(o) = v;
            } else {
                if (L.wA) o[0] = v.x;
                if (L.wB) o[1] = v.y;
            }
        }
    }
}

template <int K, bool EDGE, bool FINAL>
__device__ __forceinline__ void diffuse_wt_body(const double *__restrict__ s, double *__restrict__ d,
                                                const double *__restrict__ g, const WtLane &L, int c0, int c1,
                                                int in_lo, int in_hi, int top_reflect, int bot_reflect,
                                                double coef) {
    double2 X0[K], X1[K], X2[K], pf[3];
#pragma unroll
    for (int q = 0; q < K; ++q) X0[q] = X1[q] = X2[q] = make_double2(0.0, 0.0);
    const int i0 = c0 - K, i1 = c1 + 2 * K - 1;
    const int64_t ny = L.ny;
#pragma unroll
    for (int u = 0; u < 3; ++u) pf[u] = wt_load<EDGE>(s, (int64_t)min(max(i0 + u, in_lo), in_hi - 1) * ny, L);
    // iterations [s_lo, s_hi] have every stage active (fill ends, drain not begun)
    const int s_lo = c0 + 2 * K - 1, s_hi = c1 + K - 1;
#define WT_RUN(ST, U, I) wt_iter<K, EDGE, FINAL, ST, U>(X0, X1, X2, pf, s, d, g, L, I, c0, c1, in_lo, in_hi, top_reflect, bot_reflect, coef)
    int i = i0;
    for (; i + 3 <= i1 && i < s_lo; i += 3) {   // fill
        WT_RUN(false, 0, i); WT_RUN(false, 1, i + 1); WT_RUN(false, 2, i + 2);
    }
    for (; i + 2 <= s_hi; i += 3) {              // steady state: branch-free stages
        WT_RUN(true, 0, i); WT_RUN(true, 1, i + 1); WT_RUN(true, 2, i + 2);
    }
    for (; i + 3 <= i1; i += 3) {                // drain
        WT_RUN(false, 0, i); WT_RUN(false, 1, i + 1); WT_RUN(false, 2, i + 2);
    }
    if (i < i1) WT_RUN(false, 0, i);
    if (i + 1 < i1) WT_RUN(false, 1, i + 1);
#undef WT_RUN
}

template <int K, bool FINAL>
__global__ __launch_bounds__(256) void k_diffuse_wt(const double *__restrict__ src, double *__restrict__ dst,
                                                    const double *__restrict__ f0, int64_t field_stride, int ny,
                                                    int out_lo, int out_hi, int in_lo, int in_hi, int top_reflect,
                                                    int bot_reflect, int rows_per_chunk, int tiles_x, int chunks_y,
                                                    int n_fields, double coef, const double *__restrict__ uniform) {
    constexpr int KH = K + (K & 1);           // even halo keeps 16-B alignment
    constexpr int W = WT_COLS - 2 * KH;       // output columns per tile
    const int wave = __builtin_amdgcn_readfirstlane((int)(blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)));
    const int lane = threadIdx.x & 63;
    if (wave >= tiles_x * chunks_y * n_fields) return;
    const int tx = wave % tiles_x;
    const int ty = (wave / tiles_x) % chunks_y;
    const int f = wave / (tiles_x * chunks_y);
    if (uniform && uniform[2 * f] == uniform[2 * f + 1]) return;  // uniform plane: zero delta
    const int c0 = out_lo + ty * rows_per_chunk;
    const int c1 = min(c0 + rows_per_chunk, out_hi);
    const int x0 = tx * W;                    // first output column
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
    // reflecting boundaries or ragged columns inside the tile -> EDGE body
    const bool edge = (x0 - KH <= 0) || (x0 - KH + WT_COLS >= ny) || (ny & 1) ||
                      (top_reflect >= c0 - 3 * K - 2 && top_reflect <= c1 + 2 * K) ||
                      (bot_reflect >= c0 - 3 * K - 2 && bot_reflect <= c1 + 2 * K);
    if (edge)
        diffuse_wt_body<K, true, FINAL>(s, d, g, L, c0, c1, in_lo, in_hi, top_reflect, bot_reflect, coef);
    else
        diffuse_wt_body<K, false, FINAL>(s, d, g, L, c0, c1, in_lo, in_hi, top_reflect, bot_reflect, coef);
}

// ---------------------------------------------------------------------------
// Wave-tile, lag-1 pipeline (variant 2).  Same tile / DPP scheme as
// k_diffuse_wt, but stage q consumes stage q-1's output of the SAME iteration
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
                                        const double *__restrict__ s, double *__restrict__ d,
                                        const double *__restrict__ g, const WtLane &L, int i, int c0, int c1,
                                        int in_lo, int in_hi, int top_reflect, int bot_reflect, double coef) {
    constexpr int R = U % 3;
    double2(&UP)[K] = R == 0 ? S0 : (R == 1 ? S1 : S2);
    double2(&CN)[K] = R == 0 ? S1 : (R == 1 ? S2 : S0);
    double2(&FR)[K] = R == 0 ? S2 : (R == 1 ? S0 : S1);
    const int64_t ny = L.ny;
    FR[0] = pf[U];                                                                          // row i
    pf[U] = wt_load<EDGE>(s, (int64_t)min(max(i + PD, in_lo), in_hi - 1) * ny, L);     // row i+PD
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
                if (L.wA) *reinterpret_cast<double2 *>(o) = v;
            } else {
                if (L.wA) o[0] = v.x;
                if (L.wB) o[1] = v.y;
            }
        }
    }
}

template <int K, int PD, bool EDGE, bool FINAL, bool STEADY, int U0, int... Us>
__device__ __forceinline__ void wl_group(double2 (&S0)[K], double2 (&S1)[K], double2 (&S2)[K],
                                         double2 (&pf)[PD], double2 (&gp)[3], const double *__restrict__ s, double *__restrict__ d,
                                         const double *__restrict__ g, const WtLane &L, int i, int c0, int c1,
                                         int in_lo, int in_hi, int top_reflect, int bot_reflect, double coef) {
    wl_iter<K, PD, EDGE, FINAL, STEADY, U0>(S0, S1, S2, pf, gp, s, d, g, L, i, c0, c1, in_lo, in_hi, top_reflect,
                                        bot_reflect, coef);
    if constexpr (sizeof...(Us) > 0)
        wl_group<K, PD, EDGE, FINAL, STEADY, Us...>(S0, S1, S2, pf, gp, s, d, g, L, i + 1, c0, c1, in_lo, in_hi,
                                                top_reflect, bot_reflect, coef);
}

template <int K, int PD, bool EDGE, bool FINAL, int... Us>
__device__ __forceinline__ void diffuse_wl_loop(std::integer_sequence<int, Us...>, double2 (&S0)[K],
                                                double2 (&S1)[K], double2 (&S2)[K], double2 (&pf)[PD], double2 (&gp)[3],
                                                const double *__restrict__ s, double *__restrict__ d,
                                                const double *__restrict__ g, const WtLane &L, int c0, int c1,
                                                int in_lo, int in_hi, int top_reflect, int bot_reflect,
                                                double coef) {
    const int i0 = c0 - K + 2, i1 = c1 + K;          // iterations [i0, i1)
    const int s_lo = c0 + K, s_hi = c1 + K - 1;      // every stage active for i in [s_lo, s_hi]
#define WL_ARGS S0, S1, S2, pf, gp, s, d, g, L, i, c0, c1, in_lo, in_hi, top_reflect, bot_reflect, coef
    int i = i0;
    for (; i + PD <= i1 && i < s_lo; i += PD) wl_group<K, PD, EDGE, FINAL, false, Us...>(WL_ARGS);   // fill
    for (; i + PD - 1 <= s_hi; i += PD) wl_group<K, PD, EDGE, FINAL, true, Us...>(WL_ARGS);          // steady
    for (; i + PD <= i1; i += PD) wl_group<K, PD, EDGE, FINAL, false, Us...>(WL_ARGS);               // drain
    // tail: fewer than PD iterations, phases 0.. in order
    ((i + Us < i1 ? wl_iter<K, PD, EDGE, FINAL, false, Us>(S0, S1, S2, pf, gp, s, d, g, L, i + Us, c0, c1, in_lo,
                                                        in_hi, top_reflect, bot_reflect, coef)
                  : void()), ...);
#undef WL_ARGS
}

template <int K, int PD, bool EDGE, bool FINAL>
__device__ __forceinline__ void diffuse_wl_body(const double *__restrict__ s, double *__restrict__ d,
                                                const double *__restrict__ g, const WtLane &L, int c0, int c1,
                                                int in_lo, int in_hi, int top_reflect, int bot_reflect,
                                                double coef) {
    double2 S0[K], S1[K], S2[K], pf[PD], gp[3];
#pragma unroll
    for (int q = 0; q < K; ++q) S0[q] = S1[q] = S2[q] = make_double2(0.0, 0.0);
    const int64_t ny = L.ny;
    const int i0 = c0 - K + 2;
    // stage 0's window before the first iteration: up = row i0-2, centre = row i0-1
    S0[0] = wt_load<EDGE>(s, (int64_t)min(max(i0 - 2, in_lo), in_hi - 1) * ny, L);
    S1[0] = wt_load<EDGE>(s, (int64_t)min(max(i0 - 1, in_lo), in_hi - 1) * ny, L);
#pragma unroll
    for (int u = 0; u < PD; ++u) pf[u] = wt_load<EDGE>(s, (int64_t)min(max(i0 + u, in_lo), in_hi - 1) * ny, L);
#pragma unroll
    for (int u = 0; u < 3; ++u)   // FINAL: base rows of the first 3 output rows (i0 - K + u)
        gp[u] = FINAL && (L.wA || L.wB) ? wt_load<EDGE>(g, (int64_t)min(max(i0 - K + u, c0), c1 - 1) * ny, L)
                                        : make_double2(0.0, 0.0);
    diffuse_wl_loop<K, PD, EDGE, FINAL>(std::make_integer_sequence<int, PD>(), S0, S1, S2, pf, gp, s, d, g, L, c0, c1,
                                    in_lo, in_hi, top_reflect, bot_reflect, coef);
}

template <int K, int PD, bool FINAL>
__global__ __launch_bounds__(256) void k_diffuse_wl(const double *__restrict__ src, double *__restrict__ dst,
                                                    const double *__restrict__ f0, int64_t field_stride, int ny,
                                                    int out_lo, int out_hi, int in_lo, int in_hi, int top_reflect,
                                                    int bot_reflect, int rows_per_chunk, int tiles_x, int chunks_y,
                                                    int n_fields, double coef, const double *__restrict__ uniform) {
    constexpr int KH = K + (K & 1);
    constexpr int W = WT_COLS - 2 * KH;
    // (An XCD-contiguous tile order -- each XCD's L2 serving its tiles' shared
    // halo columns -- measured 4 % slower on 4096^2: the halo re-reads already
    // hit the die-level Infinity Cache, so plain round-robin order is kept.)
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

static int g_stencil_rows = 64;   // output rows per wave tile; 0 = auto (chunk_rows below)

// Rows per wave tile: g_stencil_rows, or (auto) the largest <= 64 that still
// yields ~4 waves per SIMD on the 1024 SIMDs -- small row bands (multi-GPU
// strong scaling) trade pipeline fill for occupancy.
static int chunk_rows(int out_rows, int tiles_x, int nf) {
    if (g_stencil_rows > 0) return g_stencil_rows;
    const int64_t want_waves = 4096;
    int r = (int)(((int64_t)out_rows * tiles_x * nf) / want_waves);
    return std::max(16, std::min(64, r));
}

template <int K>
static void launch_wt(hipStream_t st, const double *src, double *dst, const double *f0, int nf, int64_t fs,
                      int ny, int out_lo, int out_hi, int in_lo, int in_hi, int top, int bot, double coef,
                      const double *mm) {
    constexpr int KH = K + (K & 1);
    constexpr int W = WT_COLS - 2 * KH;
    const int tiles_x = (ny + W - 1) / W;
    const int rch = chunk_rows(out_hi - out_lo, tiles_x, nf);
    const int chunks_y = (out_hi - out_lo + rch - 1) / rch;
    const int waves = tiles_x * chunks_y * nf;
    if (f0)
        hipLaunchKernelGGL((k_diffuse_wt<K, true>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst, f0, fs, ny,
                           out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef, mm);
    else
        hipLaunchKernelGGL((k_diffuse_wt<K, false>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst, f0, fs, ny,
                           out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef, mm);
}

static int g_stencil_kernel = 3;  // 0 = workgroup tile (LDS), 1 = wave tile (DPP), 2/3/4 = wave tile lag-1, prefetch 3/6/9 rows

template <int K, int PD>
static void launch_wl(hipStream_t st, const double *src, double *dst, const double *f0, int nf, int64_t fs,
                      int ny, int out_lo, int out_hi, int in_lo, int in_hi, int top, int bot, double coef,
                      const double *mm) {
    constexpr int KH = K + (K & 1);
    constexpr int W = WT_COLS - 2 * KH;
    const int tiles_x = (ny + W - 1) / W;
    const int rch = chunk_rows(out_hi - out_lo, tiles_x, nf);
    const int chunks_y = (out_hi - out_lo + rch - 1) / rch;
    const int waves = tiles_x * chunks_y * nf;
    if (f0)
        hipLaunchKernelGGL((k_diffuse_wl<K, PD, true>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst, f0, fs,
                           ny, out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef, mm);
    else
        hipLaunchKernelGGL((k_diffuse_wl<K, PD, false>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst, f0, fs,
                           ny, out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef, mm);
}

template <int PD>
static void launch_wl_k(int k, hipStream_t st, const double *src, double *dst, const double *f0, int nf,
                        int64_t fs, int ny, int out_lo, int out_hi, int in_lo, int in_hi, int top, int bot,
                        double coef, const double *mm) {
#define VK_WL(KC) case KC: launch_wl<KC, PD>(st, src, dst, f0, nf, fs, ny, out_lo, out_hi, in_lo, in_hi, top, bot, coef, mm); break
    switch (k) {
        VK_WL(3); VK_WL(5); VK_WL(7); VK_WL(9); VK_WL(11); VK_WL(13); VK_WL(15);
        default: break;
    }
#undef VK_WL
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

extern "C" int vk_set_stencil_kernel(int32_t variant, int32_t rows) {
    const int prev = g_stencil_kernel;
    if (variant >= 0 && variant <= 4) g_stencil_kernel = variant;
    if (rows == 0 || (rows >= 8 && rows <= 4096)) g_stencil_rows = rows;
    return prev;
}

static int g_stencil_depth = 9;   // max substeps per HBM pass (odd; 1 = one launch per substep)

extern "C" int vk_set_stencil_depth(int32_t k) {
    const int prev = g_stencil_depth;
    if (k >= 1 && k <= 15) g_stencil_depth = k | 1;
    return prev;
}

// rows [lo, hi) of every non-uniform plane: dst <- src
__global__ __launch_bounds__(256) void k_copy_rows(const double *__restrict__ src, double *__restrict__ dst,
                                                   int64_t field_stride, int64_t off, int64_t count,
                                                   const double *__restrict__ uniform) {
    const int f = blockIdx.y;
    if (uniform && uniform[2 * f] == uniform[2 * f + 1]) return;
    const int64_t base = (int64_t)f * field_stride + off;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x)
        dst[base + i] = src[base + i];
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

extern "C" int vk_diffuse(double *field, double *work0, double *work1, int32_t n_fields,
                          int64_t field_stride, int32_t ny, int32_t row_lo, int32_t row_hi, int32_t lo_min,
                          int32_t hi_max, int32_t edge_top, int32_t edge_bot, int32_t sub_begin,
                          int32_t sub_count, int32_t n_sub, double coeff_dt, const double *uniform,
                          vk_stream_t stream) {
    if (!field || n_fields < 0 || ny <= 0 || row_lo < lo_min || row_hi > hi_max || row_lo >= row_hi ||
        sub_begin < 0 || sub_count < 0 || sub_begin + sub_count > n_sub ||
        (int64_t)hi_max * ny > field_stride) {
        vk::set_error("vk_diffuse: bad geometry");
        return VK_ERR_ARG;
    }
    if (!work0 || (n_sub > 2 && !work1)) {
        vk::set_error("vk_diffuse: work buffers required");
        return VK_ERR_ARG;
    }
    if (n_fields == 0 || sub_count == 0) return VK_OK;
    // The state after substep j lives in work[j & 1] (field after the last
    // substep).  A pass of k substeps [j, j+k) reads work[(j-1)&1] (field for
    // j == 0) and writes work[(j+k-1)&1]; k is kept ODD so the two differ.
    double *work[2] = {work0, work1};
    const int top_reflect = edge_top ? lo_min : -1;
    const int bot_reflect = edge_bot ? hi_max - 1 : 0x7fffffff;
    hipStream_t s = (hipStream_t)stream;
    const int last_in_call = sub_begin + sub_count - 1;
    int depth = g_stencil_depth | 1;   // odd
    if (depth > 15) depth = 15;
    // Pass plan: the fewest odd depths <= depth that sum to sub_count (a sum of
    // P odd numbers has the parity of P), as even as possible -- e.g. 100 =
    // 8x9 + 4x7 rather than 11x9 + a lone single-substep pass.
    int passes = (sub_count + depth - 1) / depth;
    if ((passes & 1) != (sub_count & 1)) ++passes;
    for (int j = sub_begin, left = passes; j <= last_in_call; --left) {
        const int rem = last_in_call - j + 1;   // rem has the parity of `left`
        int k = (rem + left - 1) / left;
        if ((k & 1) == 0) ++k;
        if (k > depth) k = depth;
        while (k > 1 && rem - k < left - 1) k -= 2;
        const int e = j + k - 1;     // last substep of this pass
        const int grow = last_in_call - e;
        const int lo = max(lo_min, row_lo - grow);
        const int hi = min(hi_max, row_hi + grow);
        const int in_lo = max(lo_min, lo - k), in_hi = min(hi_max, hi + k);
        const double *src = (j == 0) ? field : work[(j - 1) & 1];
        const bool final_pass = (e == n_sub - 1);
        // a pass that both starts from and ends in `field` cannot run in place
        // (neighbours would read new values): it goes through work0 + copy
        const bool in_place = final_pass && j == 0;
        double *dst = (final_pass && !in_place) ? field : (in_place ? work0 : work[e & 1]);
        const double *f0 = final_pass ? field : nullptr;
        if (k == 1) {
            dim3 grid((ny + ST_BX - 1) / ST_BX, (hi - lo + ST_RB - 1) / ST_RB, n_fields);
            hipLaunchKernelGGL(k_diffuse_substep, grid, dim3(ST_BX), 0, s, src, dst, f0, field_stride, ny, lo,
                               hi, top_reflect, bot_reflect, coeff_dt, uniform);
        } else if (g_stencil_kernel >= 2) {
            // the final pass also streams the base plane (3 rows ahead): it keeps the
            // shallow row prefetch so that it still fits 3 waves per SIMD
            auto launch = (g_stencil_kernel == 2 || f0) ? launch_wl_k<3>
                                                        : (g_stencil_kernel == 3 ? launch_wl_k<6> : launch_wl_k<9>);
            launch(k, s, src, dst, f0, n_fields, field_stride, ny, lo, hi, in_lo, in_hi, top_reflect, bot_reflect,
                   coeff_dt, uniform);
        } else if (g_stencil_kernel == 1) {
            launch_wt_k(k, s, src, dst, f0, n_fields, field_stride, ny, lo, hi, in_lo, in_hi, top_reflect,
                        bot_reflect, coeff_dt, uniform);
        } else {
            launch_tb_k(k, s, src, dst, f0, n_fields, field_stride, ny, lo, hi, in_lo, in_hi, top_reflect,
                        bot_reflect, coeff_dt, uniform);
        }
        int rc = vk::launch_check("vk_diffuse kernel");
        if (rc) return rc;
        if (in_place) {
            const int64_t count = (int64_t)(row_hi - row_lo) * ny;
            const unsigned blocks = (unsigned)std::min<int64_t>(2048, (count + 255) / 256);
            hipLaunchKernelGGL(k_copy_rows, dim3(blocks, n_fields), dim3(256), 0, s, work0, field, field_stride,
                               (int64_t)row_lo * ny, count, uniform);
            rc = vk::launch_check("k_copy_rows");
            if (rc) return rc;
        }
        j += k;
    }
    return VK_OK;
}

// ---------------------------------------------------------------------------
// uniform-plane test (diffusion_field.py:401-404: a field whose values are all
// equal gets a zero delta).  Summary per plane: sum[2f] == sum[2f+1] iff the
// owned rows hold one value (both = that value); otherwise (-inf, +inf).  The
// summary min/max-reduces across ranks (distributed.make_uniform_allreduce).
// A fixed grid of VK_UNIFORM_BLOCKS blocks per plane strides over the plane
// in 16-KiB chunks and stops at its first chunk holding a second value, so a
// non-uniform plane costs one chunk per block (a few microseconds); every
// block writes its own flag (no shared address is polled or stored to), and
// a one-block pass folds the flags into the summary.
// ---------------------------------------------------------------------------

constexpr int UN_PER_THREAD = 8;
constexpr int UN_CHUNK = 256 * UN_PER_THREAD;

__global__ __launch_bounds__(256) void k_uniform_probe(const double *__restrict__ fields, int64_t field_stride,
                                                       int64_t off, int64_t count, int32_t *__restrict__ found) {
    const int f = blockIdx.y;
    const double *p = fields + (int64_t)f * field_stride + off;
    const double v0 = p[0];
    int hit = !(v0 == v0);                       // a NaN plane is non-uniform
    for (int64_t c = blockIdx.x; !hit && c * UN_CHUNK < count; c += gridDim.x) {
        const int64_t base = c * UN_CHUNK + threadIdx.x;
        bool diff = false;
#pragma unroll
        for (int k = 0; k < UN_PER_THREAD; ++k) {
            const int64_t i = base + (int64_t)k * 256;
            if (i < count) diff |= !(p[i] == v0);
        }
        hit = __syncthreads_or(diff);
    }
    if (threadIdx.x == 0) found[(int64_t)f * gridDim.x + blockIdx.x] = hit;
}

__global__ __launch_bounds__(256) void k_uniform_finish(const double *__restrict__ fields, int64_t field_stride,
                                                        int64_t off, const int32_t *__restrict__ found,
                                                        int n_blocks, double *__restrict__ sum) {
    const int f = blockIdx.x;
    int hit = 0;
    for (int b = threadIdx.x; b < n_blocks; b += 256) hit |= found[(int64_t)f * n_blocks + b];
    hit = __syncthreads_or(hit);
    if (threadIdx.x == 0) {
        const double v0 = fields[(int64_t)f * field_stride + off];
        sum[2 * f] = hit ? -INFINITY : v0;
        sum[2 * f + 1] = hit ? INFINITY : v0;
    }
}

extern "C" int vk_field_uniform(const double *fields, int32_t n_fields, int64_t field_stride, int32_t ny,
                                int32_t row_lo, int32_t row_hi, double *summary, int32_t *scratch,
                                vk_stream_t stream) {
    if (!fields || !summary || !scratch || n_fields < 0 || n_fields > 65535 || ny <= 0 || row_lo < 0 ||
        row_hi <= row_lo || (int64_t)row_hi * ny > field_stride) {
        vk::set_error("vk_field_uniform: bad arguments");
        return VK_ERR_ARG;
    }
    if (n_fields == 0) return VK_OK;
    hipStream_t s = (hipStream_t)stream;
    const int64_t off = (int64_t)row_lo * ny;
    const int64_t count = (int64_t)(row_hi - row_lo) * ny;
    const int blocks = (int)std::min<int64_t>(VK_UNIFORM_BLOCKS, (count + UN_CHUNK - 1) / UN_CHUNK);
    hipLaunchKernelGGL(k_uniform_probe, dim3(blocks, n_fields), dim3(256), 0, s, fields, field_stride, off, count,
                       scratch);
    hipLaunchKernelGGL(k_uniform_finish, dim3(n_fields), dim3(256), 0, s, fields, field_stride, off, scratch, blocks,
                       summary);
    return vk::launch_check("k_uniform_probe");
}

// ---------------------------------------------------------------------------
// agent <-> field coupling
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_gather(const double *__restrict__ fields, int64_t field_stride,
                                                const int32_t *__restrict__ bin_lin, int64_t n,
                                                const int32_t *__restrict__ map_field,
                                                const int32_t *__restrict__ map_row, int n_map,
                                                double *__restrict__ dst, int64_t ld) {
    const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= n) return;
    const int64_t b = bin_lin[a];
    for (int i = 0; i < n_map; ++i)
        dst[(int64_t)ldc(map_row, i) * ld + a] = fields[(int64_t)ldc(map_field, i) * field_stride + b];
}

extern "C" int vk_gather(const double *fields, int64_t field_stride, const int32_t *bin_lin, int64_t n,
                         const int32_t *map_field, const int32_t *map_row, int32_t n_map, double *dst,
                         int64_t ld, vk_stream_t stream) {
    if (n < 0 || ld < n || n_map < 0 || (n > 0 && n_map > 0 && (!fields || !bin_lin || !map_field || !map_row || !dst))) {
        vk::set_error("vk_gather: bad arguments");
        return VK_ERR_ARG;
    }
    if (n == 0 || n_map == 0) return VK_OK;
    hipLaunchKernelGGL(k_gather, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, fields,
                       field_stride, bin_lin, n, map_field, map_row, n_map, dst, ld);
    return vk::launch_check("k_gather");
}

// count / (bin_volume * N_A) mol/L, to mmol/L (registry.py:179-182)
__device__ __forceinline__ double exchange_mM(int64_t count, double binvol_avogadro) {
    return ((double)count / binvol_avogadro) * 1000.0;
}

__global__ __launch_bounds__(256) void k_exchange_sorted(double *__restrict__ fields, int64_t field_stride,
                                                         const int32_t *__restrict__ occ_bin,
                                                         const int32_t *__restrict__ occ_ptr,
                                                         const int32_t *__restrict__ occ_agent, int n_occ,
                                                         const int64_t *__restrict__ counts, int64_t ld,
                                                         const int32_t *__restrict__ map_count,
                                                         const int32_t *__restrict__ map_field, int n_map,
                                                         double bva) {
    const int b = blockIdx.x * blockDim.x + threadIdx.x;
    if (b >= n_occ) return;
    const int64_t bin = occ_bin[b];
    const int k0 = occ_ptr[b], k1 = occ_ptr[b + 1];
    for (int i = 0; i < n_map; ++i) {
        double *p = fields + (int64_t)ldc(map_field, i) * field_stride + bin;
        const int64_t *cr = counts + (int64_t)ldc(map_count, i) * ld;
        double v = *p;
        for (int k = k0; k < k1; ++k) v = v + exchange_mM(cr[occ_agent[k]], bva);
        *p = v;
    }
}

extern "C" int vk_exchange_sorted(double *fields, int64_t field_stride, const int32_t *occ_bin,
                                  const int32_t *occ_ptr, const int32_t *occ_agent, int32_t n_occ,
                                  const int64_t *counts, int64_t ld, const int32_t *map_count,
                                  const int32_t *map_field, int32_t n_map, double binvol_avogadro,
                                  vk_stream_t stream) {
    if (n_occ < 0 || n_map < 0 ||
        (n_occ > 0 && n_map > 0 && (!fields || !occ_bin || !occ_ptr || !occ_agent || !counts || !map_count || !map_field))) {
        vk::set_error("vk_exchange_sorted: bad arguments");
        return VK_ERR_ARG;
    }
    if (n_occ == 0 || n_map == 0) return VK_OK;
    hipLaunchKernelGGL(k_exchange_sorted, dim3((unsigned)((n_occ + 255) / 256)), dim3(256), 0,
                       (hipStream_t)stream, fields, field_stride, occ_bin, occ_ptr, occ_agent, n_occ, counts,
                       ld, map_count, map_field, n_map, binvol_avogadro);
    return vk::launch_check("k_exchange_sorted");
}

__global__ __launch_bounds__(256) void k_exchange_atomic(double *__restrict__ fields, int64_t field_stride,
                                                         const int32_t *__restrict__ bin_lin, int64_t n,
                                                         const int64_t *__restrict__ counts, int64_t ld,
                                                         const int32_t *__restrict__ map_count,
                                                         const int32_t *__restrict__ map_field, int n_map,
                                                         double bva) {
    const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= n) return;
    const int64_t b = bin_lin[a];
    for (int i = 0; i < n_map; ++i) {
        const int64_t c = counts[(int64_t)ldc(map_count, i) * ld + a];
        if (c != 0)
            unsafeAtomicAdd(fields + (int64_t)ldc(map_field, i) * field_stride + b, exchange_mM(c, bva));
    }
}

extern "C" int vk_exchange_atomic(double *fields, int64_t field_stride, const int32_t *bin_lin, int64_t n,
                                  const int64_t *counts, int64_t ld, const int32_t *map_count,
                                  const int32_t *map_field, int32_t n_map, double binvol_avogadro,
                                  vk_stream_t stream) {
    if (n < 0 || ld < n || n_map < 0 ||
        (n > 0 && n_map > 0 && (!fields || !bin_lin || !counts || !map_count || !map_field))) {
        vk::set_error("vk_exchange_atomic: bad arguments");
        return VK_ERR_ARG;
    }
    if (n == 0 || n_map == 0) return VK_OK;
    hipLaunchKernelGGL(k_exchange_atomic, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       fields, field_stride, bin_lin, n, counts, ld, map_count, map_field, n_map,
                       binvol_avogadro);
    return vk::launch_check("k_exchange_atomic");
}

// get_bin_site: floor(loc * n / bound) as int, then Python/numpy floor-mod n.
__device__ __forceinline__ int bin_axis(double loc, int n, double bound) {
    const double v = floor(loc * n / bound);
    if (!(fabs(v) < 9.0e15)) return 0;
    int64_t i = (int64_t)v % n;
    if (i < 0) i += n;
    return (int)i;
}

__global__ __launch_bounds__(256) void k_bin_sites(const double *__restrict__ loc, int64_t n, int64_t ld, int nx,
                                                   int ny, double bx, double by, int row_offset,
                                                   int32_t *__restrict__ bin_lin, int32_t *__restrict__ ix_out) {
    const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= n) return;
    const int ix = bin_axis(loc[a], nx, bx);
    const int iy = bin_axis(loc[ld + a], ny, by);
    bin_lin[a] = (ix - row_offset) * ny + iy;
    if (ix_out) ix_out[a] = ix;
}

extern "C" int vk_bin_sites(const double *loc, int64_t n, int64_t ld, int32_t nx, int32_t ny, double bound_x,
                            double bound_y, int32_t row_offset, int32_t *bin_lin, int32_t *ix_out,
                            vk_stream_t stream) {
    if (n < 0 || ld < n || nx <= 0 || ny <= 0 || (n > 0 && (!loc || !bin_lin))) {
        vk::set_error("vk_bin_sites: bad arguments");
        return VK_ERR_ARG;
    }
    if (n == 0) return VK_OK;
    hipLaunchKernelGGL(k_bin_sites, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, loc, n,
                       ld, nx, ny, bound_x, bound_y, row_offset, bin_lin, ix_out);
    return vk::launch_check("k_bin_sites");
}
