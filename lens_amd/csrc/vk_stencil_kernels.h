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
                                        double *d, const double *g, int ny, int i,
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
                                                double *d, const double *g, int ny,
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
__global__ __launch_bounds__(TB_BX) void k_diffuse_tb(const double *__restrict__ src, double *dst,
                                                      const double *f0, int64_t field_stride, int ny,
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
    uint32_t voff;       // VK_WL_BUF_STORE: byte offset of column A in its row, out of range (store dropped) if not wA
    bool rev;            // VK_WL_ZIGZAG: this wave walks its chunk bottom-up (physical row = m - logical row)
    int m;
    bool wA, wB;         // writes its column A / B
    bool lA, rA, lB, rB; // reflect flags (EDGE tiles only)
};

// Physical row of logical row x, clamped into the pass's input rows [lo, hi).
__device__ __forceinline__ int64_t wl_row(const WtLane &L, int x, int lo, int hi) {
    const int r = L.rev ? L.m - x : x;
    return (int64_t)min(max(r, lo), hi - 1);
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

// VK_WL_RING (variant 12/13): stage 0 reads its three rows straight from the
// prefetch ring, which then holds PD + 3 rows (up, centre, fresh and PD in
// flight), and the loop is unrolled by that ring length.  Without it the ring
// (PD slots) and the stage-0 window (3 slots) rotate with different periods, so
// the register allocator closes each unrolled group with copies of the
// in-flight rows -- and a vmcnt(0) before them, which drains every load (and
// streaming store) once per group of PD rows.
#ifdef VK_WL_RING
constexpr int wl_ring(int PD) { return PD + 3; }
constexpr bool WL_RING = true;
#else
constexpr int wl_ring(int PD) { return PD; }
constexpr bool WL_RING = false;
#endif

// PD = rows prefetched ahead in VGPRs (a multiple of 3: the slot roles rotate with period 3)
template <int K, int PD, bool EDGE, bool FINAL, bool FAST, bool SC, bool STEADY, int U>
__device__ __forceinline__ void wl_iter(double2 (&S0)[K], double2 (&S1)[K], double2 (&S2)[K], double2 (&pf)[wl_ring(PD)], double2 (&gp)[3],
                                        const double *__restrict__ s, double *d,
                                        const double *g, const WtLane &L, int i, int c0, int c1,
                                        int in_lo, int in_hi, int top_reflect, int bot_reflect, double coef,
                                        double c4) {
    constexpr int R = U % 3;
    double2(&UP)[K] = R == 0 ? S0 : (R == 1 ? S1 : S2);
    double2(&CN)[K] = R == 0 ? S1 : (R == 1 ? S2 : S0);
    double2(&FR)[K] = R == 0 ? S2 : (R == 1 ? S0 : S1);
    const int64_t ny = L.ny;
#ifdef VK_WL_BUF_STORE
    // keep each iteration's load, stages and store in program order: with the
    // stores branch-free, a steady group of PD iterations is one basic block, and
    // the scheduler would otherwise cluster its PD loads at the end of the block
    __builtin_amdgcn_sched_barrier(0);
#endif
    constexpr int NR = wl_ring(PD);
    if constexpr (WL_RING) {
        // row j lives in slot (j - i0) mod NR; U = (i - i0) mod NR.  Row i+PD goes
        // to the slot of row i-3, whose last use (as stage 0's up row) was iteration i-1
        pf[(U + PD) % NR] = wt_load<EDGE>(s, wl_row(L, i + PD, in_lo, in_hi) * ny, L);
    } else {
        FR[0] = pf[U];                                                                      // row i
        pf[U] = wt_load<EDGE>(s, wl_row(L, i + PD, in_lo, in_hi) * ny, L);             // row i+PD
    }
    const int r_out = i - K;
    const bool row_ok = STEADY || (r_out >= c0 && r_out < c1);
    double2 base = make_double2(0.0, 0.0);
    if (FINAL && !FAST) {   // base row r_out arrived 3 iterations ago; fetch row r_out+3 (clamped into the chunk)
        base = gp[R];
        if (L.wA || L.wB) gp[R] = wt_load<EDGE>(g, (int64_t)min(max(r_out + 3, c0), c1 - 1) * ny, L);
    }
#pragma unroll
    for (int q = 0; q < K; ++q) {
        // stage q is useful for rows [c0-(K-1-q), c1+(K-1-q)), i.e. i in [c0-K+2+2q, c1+K)
        if (!STEADY && (i < c0 - K + 2 + 2 * q || i >= c1 + K)) continue;
        const int r = i - 1 - q;
        const bool ring0 = WL_RING && q == 0;
        const double2 cen = ring0 ? pf[(U + NR - 1) % NR] : CN[q];
        const double2 up = (EDGE && r == top_reflect) ? cen : (ring0 ? pf[(U + NR - 2) % NR] : UP[q]);
        const double2 dn = (EDGE && r == bot_reflect) ? cen : (ring0 ? pf[U % NR] : FR[q]);
        double leftA = dpp_from_lane_below(cen.y), rightB = dpp_from_lane_above(cen.x);
        double rightA = cen.y, leftB = cen.x;
        if (EDGE) {
            leftA = L.lA ? cen.x : leftA;
            rightA = L.rA ? cen.x : rightA;
            leftB = L.lB ? cen.y : leftB;
            rightB = L.rB ? cen.y : rightB;
        }
        double2 v;
        if (FAST && SC) {
            // scaled tolerance mode: stage q carries the field divided by c4^q
            // (c4 = 1 - 4coef), so c4*c + coef*sum becomes t + (coef/c4)*sum -- 4 FP64
            // ops per cell; the last stage multiplies c4^K back in.  Here coef holds
            // coef/c4 and c4 holds c4^K (diffuse_wl_tile)
            const double sA = (up.x + dn.x) + (leftA + rightA);
            const double sB = (up.y + dn.y) + (leftB + rightB);
            v = make_double2(fma(coef, sA, cen.x), fma(coef, sB, cen.y));
            if (q + 1 == K) v = make_double2(c4 * v.x, c4 * v.y);
        } else if (FAST) {
            // tolerance mode: c + coef*(N+S+E+W-4c) = fma(coef, (N+S)+(E+W), (1-4coef)*c),
            // 5 FP64 ops per cell instead of 6
            const double sA = (up.x + dn.x) + (leftA + rightA);
            const double sB = (up.y + dn.y) + (leftB + rightB);
            v = make_double2(fma(coef, sA, c4 * cen.x), fma(coef, sB, c4 * cen.y));
        } else {
            const double lapA = ((fma(-4.0, cen.x, up.x + leftA)) + rightA) + dn.x;
            const double lapB = ((fma(-4.0, cen.y, up.y + leftB)) + rightB) + dn.y;
            v = make_double2(cen.x + coef * lapA, cen.y + coef * lapB);
        }
        if (q + 1 < K) {
            FR[q + 1] = v;
        } else if (row_ok) {
            if (FINAL && !FAST) v = make_double2(base.x + (v.x - base.x), base.y + (v.y - base.y));
            const int64_t r_phys = L.rev ? L.m - r_out : r_out;
            double *o = d + r_phys * ny + L.cA;
            if (!EDGE) {
#ifdef VK_WL_BUF_STORE
                // Branch-free store: lanes that do not write carry an out-of-range
                // offset and the buffer unit drops their store.  With no exec branch
                // around the store, the compiler's vmcnt bookkeeping counts every
                // iteration's store, so a row load is awaited only PD rows after its
                // issue (a masked store made it wait as if no store were in flight:
                // about PD/2 rows of lookahead).  aux 2 = nt (streaming store).
                (void)o;
                typedef int i4v __attribute__((ext_vector_type(4)));
                const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                    (void *)(d + r_phys * ny), 0, (int)(ny * 8), 0x00020000);
                __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i4v, v), rs, (int)L.voff, 0, 2);
#else
                if (L.wA) wl_store(o, v);
#endif
            } else {
                if (L.wA) o[0] = v.x;
                if (L.wB) o[1] = v.y;
            }
        }
    }
}

template <int K, int PD, bool EDGE, bool FINAL, bool FAST, bool SC, bool STEADY, int U0, int... Us>
__device__ __forceinline__ void wl_group(double2 (&S0)[K], double2 (&S1)[K], double2 (&S2)[K],
                                         double2 (&pf)[wl_ring(PD)], double2 (&gp)[3], const double *__restrict__ s, double *d,
                                         const double *g, const WtLane &L, int i, int c0, int c1,
                                         int in_lo, int in_hi, int top_reflect, int bot_reflect, double coef,
                                         double c4) {
    wl_iter<K, PD, EDGE, FINAL, FAST, SC, STEADY, U0>(S0, S1, S2, pf, gp, s, d, g, L, i, c0, c1, in_lo, in_hi,
                                                  top_reflect, bot_reflect, coef, c4);
    if constexpr (sizeof...(Us) > 0)
        wl_group<K, PD, EDGE, FINAL, FAST, SC, STEADY, Us...>(S0, S1, S2, pf, gp, s, d, g, L, i + 1, c0, c1, in_lo,
                                                          in_hi, top_reflect, bot_reflect, coef, c4);
}

template <int K, int PD, bool EDGE, bool FINAL, bool FAST, bool SC, int... Us>
__device__ __forceinline__ void diffuse_wl_loop(std::integer_sequence<int, Us...>, double2 (&S0)[K],
                                                double2 (&S1)[K], double2 (&S2)[K], double2 (&pf)[wl_ring(PD)], double2 (&gp)[3],
                                                const double *__restrict__ s, double *d,
                                                const double *g, const WtLane &L, int c0, int c1,
                                                int in_lo, int in_hi, int top_reflect, int bot_reflect,
                                                double coef, double c4) {
    const int i0 = c0 - K + 2, i1 = c1 + K;          // iterations [i0, i1)
    const int s_lo = c0 + K, s_hi = c1 + K - 1;      // every stage active for i in [s_lo, s_hi]
#define WL_ARGS S0, S1, S2, pf, gp, s, d, g, L, i, c0, c1, in_lo, in_hi, top_reflect, bot_reflect, coef, c4
    constexpr int NU = wl_ring(PD);                  // iterations per unrolled group
    int i = i0;
    for (; i + NU <= i1 && i < s_lo; i += NU) wl_group<K, PD, EDGE, FINAL, FAST, SC, false, Us...>(WL_ARGS);   // fill
#ifdef VK_WL_BUF_STORE
    // enter the steady loop with no memory operation in flight, so that the
    // compiler's wait counts at its header come from the loop's own (branch-free)
    // iterations and not from the fill phase's conditional stores
    if (!EDGE) __builtin_amdgcn_s_waitcnt(0x0F70);   // vmcnt(0)
#endif
    for (; i + NU - 1 <= s_hi; i += NU) wl_group<K, PD, EDGE, FINAL, FAST, SC, true, Us...>(WL_ARGS);          // steady
    for (; i + NU <= i1; i += NU) wl_group<K, PD, EDGE, FINAL, FAST, SC, false, Us...>(WL_ARGS);               // drain
    // tail: fewer than NU iterations, phases 0.. in order
    ((i + Us < i1 ? wl_iter<K, PD, EDGE, FINAL, FAST, SC, false, Us>(S0, S1, S2, pf, gp, s, d, g, L, i + Us, c0, c1,
                                                              in_lo, in_hi, top_reflect, bot_reflect, coef, c4)
                  : void()), ...);
#undef WL_ARGS
}

template <int K, int PD, bool EDGE, bool FINAL, bool FAST, bool SC>
__device__ __forceinline__ void diffuse_wl_body(const double *__restrict__ s, double *d,
                                                const double *g, const WtLane &L, int c0, int c1,
                                                int in_lo, int in_hi, int top_reflect, int bot_reflect,
                                                double coef, double c4) {
    constexpr int NR = wl_ring(PD);
    double2 S0[K], S1[K], S2[K], pf[NR], gp[3];
#pragma unroll
    for (int q = 0; q < K; ++q) S0[q] = S1[q] = S2[q] = make_double2(0.0, 0.0);
    const int64_t ny = L.ny;
    const int i0 = c0 - K + 2;
    // stage 0's window before the first iteration: up = row i0-2, centre = row i0-1
    // (ring: slots NR-2 and NR-1)
    double2 &w_up = WL_RING ? pf[NR - 2] : S0[0];
    double2 &w_cn = WL_RING ? pf[NR - 1] : S1[0];
    w_up = wt_load<EDGE>(s, wl_row(L, i0 - 2, in_lo, in_hi) * ny, L);
    w_cn = wt_load<EDGE>(s, wl_row(L, i0 - 1, in_lo, in_hi) * ny, L);
#pragma unroll
    for (int u = 0; u < PD; ++u) pf[u] = wt_load<EDGE>(s, wl_row(L, i0 + u, in_lo, in_hi) * ny, L);
#pragma unroll
    for (int u = 0; u < 3; ++u)   // FINAL: base rows of the first 3 output rows (i0 - K + u)
        gp[u] = FINAL && !FAST && (L.wA || L.wB)
                    ? wt_load<EDGE>(g, (int64_t)min(max(i0 - K + u, c0), c1 - 1) * ny, L)
                    : make_double2(0.0, 0.0);
    diffuse_wl_loop<K, PD, EDGE, FINAL, FAST, SC>(std::make_integer_sequence<int, NR>(), S0, S1, S2, pf, gp, s, d, g, L,
                                              c0, c1, in_lo, in_hi, top_reflect, bot_reflect, coef, c4);
}

// FAST = tolerance mode (vk_set_stencil_mode(1)): FMA-contracted arithmetic and a
// final pass without the base re-read; within ~1e-14 relative of the exact mode.
template <int K, int PD, bool FINAL, bool FAST = false>
__device__ __forceinline__ void diffuse_wl_tile(const double *__restrict__ src, double *dst,
                                                const double *f0, int64_t field_stride, int ny,
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
#ifdef VK_WL_ZIGZAG
    // the 4 waves of a workgroup take 4 vertically adjacent chunks of one column
    // tile, odd chunks walked bottom-up: each chunk boundary's halo rows are then
    // read by both neighbours at about the same time (both at their start or both
    // at their end), mostly on one CU
    const int ty = wave % chunks_y;
    const int tx = (wave / chunks_y) % tiles_x;
#else
    const int tx = wave % tiles_x;
    const int ty = (wave / tiles_x) % chunks_y;
#endif
    const int f = wave / (tiles_x * chunks_y);
    if (uniform && uniform[2 * f] == uniform[2 * f + 1]) return;
    const int c0 = out_lo + ty * rows_per_chunk;
    const int c1 = min(c0 + rows_per_chunk, out_hi);
    const int x0 = tx * W;
    WtLane L;
    L.ny = ny;
    L.rev = false;
    L.m = 0;
    L.cA = x0 - KH + 2 * lane;
    const int cB = L.cA + 1;
    L.wA = lane >= KH / 2 && lane < 64 - KH / 2 && L.cA < ny;
    L.wB = lane >= KH / 2 && lane < 64 - KH / 2 && cB < ny;
    L.voff = L.wA ? (uint32_t)L.cA * 8u : 0x80000000u;
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
    const double c4 = 1.0 - 4.0 * coef;      // FAST only
#ifdef VK_WL_ZIGZAG
    // only the tolerance mode: (N + S) + (E + W) is symmetric in N and S, so a
    // bottom-up walk gives the same bits (the exact mode's order is not)
    L.rev = FAST && !edge && (ty & 1);
    L.m = c0 + c1 - 1;
#endif
    if constexpr (FAST) {
        // the scaled form while c4^-K stays far from overflow (|c4| >= 1e-3, i.e.
        // coef not within 2.5e-4 of 1/4; coef = 0 gives the identity exactly)
        if (fabs(c4) >= 1e-3) {
            const double q = coef / c4;
            double cK = 1.0;
#pragma unroll
            for (int k = 0; k < K; ++k) cK *= c4;
            if (edge)
                diffuse_wl_body<K, PD, true, FINAL, FAST, true>(s, d, g, L, c0, c1, in_lo, in_hi, top_reflect,
                                                                bot_reflect, q, cK);
            else
                diffuse_wl_body<K, PD, false, FINAL, FAST, true>(s, d, g, L, c0, c1, in_lo, in_hi, top_reflect,
                                                                 bot_reflect, q, cK);
            return;
        }
    }
    if (edge)
        diffuse_wl_body<K, PD, true, FINAL, FAST, false>(s, d, g, L, c0, c1, in_lo, in_hi, top_reflect, bot_reflect,
                                                         coef, c4);
    else
        diffuse_wl_body<K, PD, false, FINAL, FAST, false>(s, d, g, L, c0, c1, in_lo, in_hi, top_reflect,
                                                          bot_reflect, coef, c4);
}

// Aliasing: the FINAL pass writes the field it also reads as the base plane
// (dst == f0, vk_diffuse), so only the source plane is __restrict__; each base
// load feeds the store of the same cell, later in program order.
#define VK_WL_PARAMS                                                                                           \
    const double *__restrict__ src, double *dst, const double *f0, int64_t field_stride, \
        int ny, int out_lo, int out_hi, int in_lo, int in_hi, int top_reflect, int bot_reflect, int rows_per_chunk, \
        int tiles_x, int chunks_y, int n_fields, double coef, const double *__restrict__ uniform
#define VK_WL_ARGS                                                                                             \
    src, dst, f0, field_stride, ny, out_lo, out_hi, in_lo, in_hi, top_reflect, bot_reflect, rows_per_chunk,      \
        tiles_x, chunks_y, n_fields, coef, uniform

#ifndef VK_WL_WAVES_ATTR
#define VK_WL_WAVES_ATTR
#endif
template <int K, int PD, bool FINAL, bool FAST = false>
__global__ __launch_bounds__(256) VK_WL_WAVES_ATTR void k_diffuse_wl(VK_WL_PARAMS) {
    diffuse_wl_tile<K, PD, FINAL, FAST>(VK_WL_ARGS);
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
