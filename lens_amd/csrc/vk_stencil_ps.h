// Tolerance-mode fused stencil passes in pair-sum form (variant 20, the tolerance-mode
// default), instantiated by vk_stencil_ps*.hip.  diffusion_field.py:385-394 advances every cell by
// f += coef * (N + S + E + W - 4C); the exact mode reproduces scipy's
// convolve rounding (vk_stencil_kernels.h).  The tolerance mode only has to
// stay within 1e-13 of it, so it is free to regroup the four neighbours:
//
//     N + S + E + W  =  (W + N) + (S + E)
//
// and the pair d(r, c) = f(r+1, c) + f(r, c+1) is the S+E pair of cell (r, c)
// AND the W+N pair of cell (r+1, c+1).  Each pair is therefore added once and
// used twice: a cell-substep costs two adds and one fma (3 FP64 ops, was 4),
//
//     t' = fma(coef/c4, d(r-1, c-1) + d(r, c), t)
//
// on the field carried rescaled by c4^-stage (c4 = 1 - 4coef, the last stage
// multiplies c4^K back in), or fma(coef, ., c4*C) while |c4| < 1e-3.
//
// Layout: as variant 6 -- one wavefront = one tile of 64*C columns (C
// adjacent columns per lane), K substeps fused per pass as a lag-1 software
// pipeline over the rows (stage q computes row i-1-q at iteration i).  A stage
// keeps two rows of registers: its centre row and the d row above it.  Per
// stage and row a lane needs two doubles from its neighbours (the centre of
// the lane above, the last d of the lane below) over DPP wave shifts.
//
// Pipeline shape (no per-stage tests in the loop):
//   - fill: the first 2K-1 iterations of a chunk, unrolled at compile time,
//     stage q joining at iteration 2q (one iteration early, for its first d row);
//   - steady: exactly one iteration per output row, every stage active and
//     every row stored, unrolled by the prefetch ring length (PD + 2 rows:
//     stage 0 reads its rows in place, so no register copies).
//
// Reflecting edges (Neumann, ghost = edge value) are ghost cells: after each
// stage the lane holding column -1 (or ny) copies column 0's (ny-1's) value,
// and at the reflected rows the missing pair is formed from the row itself.
// The bits of a cell therefore do not depend on the tile or chunk that
// computes it: whole planes and row bands stay bit-identical.
#pragma once

#include "vk_stencil_kernels.h"

namespace vk_ps {

struct PsLane {
    int cA;             // first column of this lane
    int ny;
    int64_t ny64;
    uint32_t loff;      // byte offset of column cA in its row (out of range left of the plane: loads 0)
    uint32_t voff;      // the same for stores; out of range (store dropped) if the lane writes nothing
    uint32_t wmask;     // edge tiles: bit j = column cA+j is written
    uint64_t mlast[4];  // lane masks: column ny-1 at position j of the lane (its E neighbour is itself)
    uint64_t mgl;       // lane mask: the lane holds the left ghost column -1 (at j = C-1)
};

typedef int i4v __attribute__((ext_vector_type(4)));
typedef double dv2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const double *row, int ny) {
    // same descriptor word 3 as the variant-13 buffer stores of round 3
    return __builtin_amdgcn_make_buffer_rsrc((void *)row, 0, ny * 8, 0x00020000);
}

// CL = the general edge body (a row width the 16-B accesses cannot tile, a plane
// one tile wide, or a reflected row in reach): columns clamped per element and
// stores masked per column.  Otherwise 16-B buffer accesses: a lane left or
// right of the plane loads zeros (its columns are halo) and stores nothing.
// CP: bit 0 = streaming (nt) loads (A/B only), bit 1 = plain (cached) stores -- the 10-deep
// pass's choice when its planes fit the MALL (vk_stencil_ps10.hip); 0 = plain loads and
// streaming stores, the default
template <int C, bool CL, int CP = 0>
__device__ __forceinline__ void ps_load(double (&out)[C], const double *__restrict__ row, const PsLane &L) {
    if constexpr (!CL) {
        const __amdgpu_buffer_rsrc_t rs = row_rsrc(row, L.ny);
#pragma unroll
        for (int j = 0; j < C; j += 2) {
            const i4v x = __builtin_amdgcn_raw_buffer_load_b128(rs, (int)(L.loff + 8u * j), 0, (CP & 1) ? 2 : 0);
            const double2 y = __builtin_bit_cast(double2, x);
            out[j] = y.x;
            out[j + 1] = y.y;
        }
    } else {
#pragma unroll
        for (int j = 0; j < C; ++j) out[j] = row[min(max(L.cA + j, 0), L.ny - 1)];
    }
}

template <int C, bool CL, int CP = 0>
__device__ __forceinline__ void ps_store(double *row, const double (&v)[C], const PsLane &L) {
    if constexpr (!CL) {
        // branch-free: a lane that does not write carries an out-of-range offset
        // and the buffer unit drops its store (aux 2 = streaming / nt)
        const __amdgpu_buffer_rsrc_t rs = row_rsrc(row, L.ny);
#pragma unroll
        for (int j = 0; j < C; j += 2) {
            const double2 y = make_double2(v[j], v[j + 1]);
            __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(i4v, y), rs, (int)(L.voff + 8u * j), 0,
                                                   (CP & 2) ? 0 : 2);
        }
    } else {
#pragma unroll
        for (int j = 0; j < C; ++j)
            if ((L.wmask >> j) & 1) row[L.cA + j] = v[j];
    }
}

// One stage of one iteration: cn = input row r, fr = input row r+1, dold =
// d(r-1) of this lane's columns; writes dnew = d(r) and the output row r.
// Edge kinds (compile time, so interior tiles carry none of it):
//   GL  the left edge: the lane holding column -1 forms d(r, -1) from column 0's
//       next-row value (the ghost column equals column 0 at every stage);
//   GR  the right edge: the E neighbour of column ny-1 is itself;
//   EY  a reflected row in reach: at the top row the pair above is the row's own
//       (f(r, c) + f(r, c+1)), at the bottom row so is the pair below.
// Per-lane select m ? a : b for a wave-wide lane mask m (SGPR pair).  Written
// as v_cndmask in asm because the compiler otherwise folds `sel ? dpp(x) : y`
// into a DPP mov executed under exec = sel -- and a DPP read from a lane
// outside exec returns 0 (bound_ctrl): the edge ghosts read zeros.  (Pinning
// the DPP result with an empty volatile asm instead cost the edge body its
// schedule: 204 VGPRs.)
__device__ __forceinline__ double ps_sel(uint64_t m, double a, double b) {
    const int2 ai = __builtin_bit_cast(int2, a), bi = __builtin_bit_cast(int2, b);
    int2 r;
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r.x) : "v"(bi.x), "v"(ai.x), "s"(m));
    asm("v_cndmask_b32 %0, %1, %2, %3" : "=v"(r.y) : "v"(bi.y), "v"(ai.y), "s"(m));
    return __builtin_bit_cast(double, r);
}

template <int C, bool GL, bool GR, bool EY, bool SC>
__device__ __forceinline__ void ps_stage(const double (&cn)[C], const double (&fr)[C], const double (&dold)[C],
                                         double (&dnew)[C], double (&v)[C], bool top, bool bot, bool first,
                                         const PsLane &L, double coef, double c4) {
    const double right = dpp_from_lane_above(cn[0]);          // f(r, cA + C)
    double e[C];                                                // E neighbours: f(r, c+1)
#pragma unroll
    for (int j = 0; j < C; ++j) {
        e[j] = j + 1 < C ? cn[j + 1] : right;
        if (GR) e[j] = ps_sel(L.mlast[j], cn[j], e[j]);
    }
    double s_[C];                                               // S neighbours: f(r+1, c)
#pragma unroll
    for (int j = 0; j < C; ++j) s_[j] = fr[j];
    // the ghost column of stage 0's input (loaded: zero) -- later stages receive
    // it fixed from the stage before
    if (GL && first) s_[C - 1] = ps_sel(L.mgl, dpp_from_lane_above(fr[0]), fr[C - 1]);
    double h[C];                                                // f(r, c) + f(r, c+1): the pair at a reflected row
    if (EY) {
#pragma unroll
        for (int j = 0; j < C; ++j) h[j] = cn[j] + e[j];   // (the ghost column's cn is column 0's)
    }
#pragma unroll
    for (int j = 0; j < C; ++j) dnew[j] = (EY && bot) ? h[j] : s_[j] + e[j];
    double dp[C];
#pragma unroll
    for (int j = 0; j < C; ++j) dp[j] = (EY && top) ? h[j] : dold[j];
    const double left = dpp_from_lane_below(dp[C - 1]);        // d(r-1, cA-1): no select follows
#pragma unroll
    for (int j = 0; j < C; ++j) {
        const double s = (j == 0 ? left : dp[j - 1]) + dnew[j];
        v[j] = SC ? fma(coef, s, cn[j]) : fma(coef, s, c4 * cn[j]);
    }
    if (GL) v[C - 1] = ps_sel(L.mgl, dpp_from_lane_above(v[0]), v[C - 1]);   // the ghost column, for the next stage
}

template <int K, int PD, int C>
struct PsState {
    static constexpr int NR = PD + 2;      // stage-0 ring: rows i-1, i and PD in flight
    double ring[NR][C];
    double Wa[K][C], Wb[K][C];             // stage q >= 1: centre / fresh rows, roles swap each iteration
    double Da[K][C], Db[K][C];             // d rows, double-buffered the same way
};

struct PsArgs {
    const double *s;
    double *d;
    int in_lo, in_hi, top, bot;
    double coef, c4, cK;
};

__device__ __forceinline__ int64_t clamp_row(int r, int lo, int hi) { return (int64_t)min(max(r, lo), hi - 1); }

// Iteration i at ring phase U (row i sits in ring slot U): prefetch row i+PD,
// run stages [0, ACT), store row i-K if STORE.
template <int K, int PD, int C, bool GL, bool GR, bool EY, bool SC, int CP, int ACT, bool STORE, int U>
__device__ __forceinline__ void ps_iter(PsState<K, PD, C> &S, const PsArgs &A, const PsLane &L, int i) {
    constexpr int NR = PD + 2;
    constexpr int P = U & 1;
    // keep iterations in program order: the scheduler would otherwise hoist the
    // unrolled group's row loads (and their registers) to its top
    __builtin_amdgcn_sched_barrier(0);
    double r0c[C], r0f[C];                 // stage 0's rows i-1 and i
    ps_load<C, GL && GR && EY, CP>(S.ring[(U + PD) % NR], A.s + clamp_row(i + PD, A.in_lo, A.in_hi) * L.ny64, L);
#pragma unroll
    for (int j = 0; j < C; ++j) {
        r0c[j] = S.ring[(U + NR - 1) % NR][j];
        r0f[j] = S.ring[U][j];
    }
#pragma unroll
    for (int q = 0; q < ACT; ++q) {
        const int r = i - 1 - q;
        const double(&cn)[C] = q == 0 ? r0c : (P == 0 ? S.Wa[q] : S.Wb[q]);
        const double(&fr)[C] = q == 0 ? r0f : (P == 0 ? S.Wb[q] : S.Wa[q]);
        const double(&dold)[C] = P == 0 ? S.Da[q] : S.Db[q];
        double(&dnew)[C] = P == 0 ? S.Db[q] : S.Da[q];
        double v[C];
        ps_stage<C, GL, GR, EY, SC>(cn, fr, dold, dnew, v, EY && r == A.top, EY && r == A.bot, q == 0, L, A.coef,
                                    A.c4);
        if (q + 1 < K) {
            double(&nx)[C] = P == 0 ? S.Wb[q + 1] : S.Wa[q + 1];
#pragma unroll
            for (int j = 0; j < C; ++j) nx[j] = v[j];
        } else if (STORE) {
            if (SC) {
#pragma unroll
                for (int j = 0; j < C; ++j) v[j] *= A.cK;
            }
            ps_store<C, GL && GR && EY, CP>(A.d + (int64_t)(i - K) * L.ny64, v, L);
        }
    }
}

template <int K, int PD, int C, bool GL, bool GR, bool EY, bool SC, int CP, int T>
__device__ __forceinline__ void ps_fill(PsState<K, PD, C> &S, const PsArgs &A, const PsLane &L, int is) {
    if constexpr (T < 2 * K - 1) {
        constexpr int ACT = T / 2 + 1 < K ? T / 2 + 1 : K;
        ps_iter<K, PD, C, GL, GR, EY, SC, CP, ACT, false, T % (PD + 2)>(S, A, L, is + T);
        ps_fill<K, PD, C, GL, GR, EY, SC, CP, T + 1>(S, A, L, is);
    }
}

// The last (i1 - i) < NR iterations, nested (iteration u runs only if u-1 ran),
// so that no state has to be merged across a skipped iteration: a flat list of
// guarded iterations keeps both versions of every row live and costs ~60 VGPRs.
template <int K, int PD, int C, bool GL, bool GR, bool EY, bool SC, int CP, int PH, int u>
__device__ __forceinline__ void ps_tail(PsState<K, PD, C> &S, const PsArgs &A, const PsLane &L, int i, int n) {
    constexpr int NR = PD + 2;
    if constexpr (u < NR - 1) {
        if (u < n) {
            ps_iter<K, PD, C, GL, GR, EY, SC, CP, K, true, (PH + u) % NR>(S, A, L, i + u);
            ps_tail<K, PD, C, GL, GR, EY, SC, CP, PH, u + 1>(S, A, L, i, n);
        }
    }
}

template <int K, int PD, int C, bool GL, bool GR, bool EY, bool SC, int CP, int... Us>
__device__ __forceinline__ void ps_steady(std::integer_sequence<int, Us...>, PsState<K, PD, C> &S, const PsArgs &A,
                                          const PsLane &L, int i, int i1) {
    constexpr int NR = PD + 2;
    constexpr int PH = (2 * K - 1) % NR;    // ring phase of the first steady iteration
    for (; i + NR <= i1; i += NR) (ps_iter<K, PD, C, GL, GR, EY, SC, CP, K, true, (PH + Us) % NR>(S, A, L, i + Us), ...);
    ps_tail<K, PD, C, GL, GR, EY, SC, CP, PH, 0>(S, A, L, i, i1 - i);
}

template <int K, int PD, int C, bool GL, bool GR, bool EY, bool SC, int CP>
__device__ __forceinline__ void ps_body(const PsArgs &A, const PsLane &L, int c0, int c1) {
    constexpr int NR = PD + 2;
    PsState<K, PD, C> S;
#pragma unroll
    for (int q = 0; q < K; ++q)
#pragma unroll
        for (int j = 0; j < C; ++j) S.Wa[q][j] = S.Wb[q][j] = S.Da[q][j] = S.Db[q][j] = 0.0;
    // iteration `is` = c0-K+1 is stage 0's d-only step (d of row c0-K for its
    // first useful row c0-K+1); it reads row is-1 from slot NR-1, row is from slot 0
    const int is = c0 - K + 1;
    ps_load<C, GL && GR && EY, CP>(S.ring[NR - 1], A.s + clamp_row(is - 1, A.in_lo, A.in_hi) * L.ny64, L);
#pragma unroll
    for (int u = 0; u < PD; ++u)
        ps_load<C, GL && GR && EY, CP>(S.ring[u], A.s + clamp_row(is + u, A.in_lo, A.in_hi) * L.ny64, L);
    ps_fill<K, PD, C, GL, GR, EY, SC, CP, 0>(S, A, L, is);
    // steady: i = c0+K .. c1+K-1, one stored row each (rows c0 .. c1-1)
    ps_steady<K, PD, C, GL, GR, EY, SC, CP>(std::make_integer_sequence<int, NR>(), S, A, L, c0 + K, c1 + K);
}

// The stencil work of one wave: its tile of plane f, output rows [c0, c1)
template <int K, int PD, int C, bool SC, int CP, int KH, int W>
__device__ __forceinline__ void ps_plane(const double *__restrict__ src, double *dst, int64_t field_stride, int ny,
                                         int in_lo, int in_hi, int top_reflect, int bot_reflect, double coef,
                                         double c4, double cK, int f, int x0, int c0, int c1, int lane) {
    PsLane L;
    L.ny = ny;
    L.ny64 = ny;
    L.cA = x0 - KH + C * lane;
    const bool writer_lane = lane >= KH / C && lane < 64 - KH / C;
    L.wmask = 0;
#pragma unroll
    for (int j = 0; j < C; ++j)
        if (writer_lane && L.cA + j >= 0 && L.cA + j < ny) L.wmask |= 1u << j;
#pragma unroll
    for (int j = 0; j < C; ++j) L.mlast[j] = __builtin_amdgcn_ballot_w64(L.cA + j == ny - 1);
    L.mgl = __builtin_amdgcn_ballot_w64(L.cA + C - 1 == -1);
    L.loff = (uint32_t)L.cA * 8u;
    L.voff = (writer_lane && L.cA >= 0 && L.cA + C <= ny) ? (uint32_t)L.cA * 8u : 0x80000000u;
    PsArgs A;
    A.s = src + (int64_t)f * field_stride;
    A.d = dst + (int64_t)f * field_stride;
    A.in_lo = in_lo;
    A.in_hi = in_hi;
    A.top = top_reflect;
    A.bot = bot_reflect;
    A.coef = coef;
    A.c4 = c4;
    A.cK = cK;
    // edge kinds in reach of this tile's rows and columns
    const bool gl = x0 - KH <= 0;
    const bool gr = x0 - KH + 64 * C >= ny;
    const bool ey = (top_reflect >= c0 - 2 * K - 2 && top_reflect <= c1 + 2 * K) ||
                    (bot_reflect >= c0 - 2 * K - 2 && bot_reflect <= c1 + 2 * K);
    // Three bodies: interior tiles; side tiles (a plane side in reach, no reflected
    // row: 16-B accesses, both ghost fixes -- a no-op on the side the tile does not
    // touch; C4 1.361 -> 1.337 ms per step, profiles/r05/r05ac/); and one general edge
    // body (every edge kind, clamped columns: reflected rows, planes one tile wide,
    // odd widths).  167 VGPRs (3 waves per SIMD); separate left / right bodies, or a
    // fourth body for reflected rows alone (171), take it to 2 waves per SIMD.  The
    // unscaled form (coef ~ 1/4) runs the general body everywhere.
    if (!SC || ey || (gl && gr) || (ny % C) != 0)
        ps_body<K, PD, C, true, true, true, SC, CP>(A, L, c0, c1);
    else if constexpr (SC) {
        if (gl || gr)
            ps_body<K, PD, C, true, true, false, SC, CP>(A, L, c0, c1);
        else
            ps_body<K, PD, C, false, false, false, SC, CP>(A, L, c0, c1);
    }
}

// KHO > 0: that many halo columns per side instead of the fewest whole lanes >= K
// (KHO = 16: 96 written columns, every tile's rows 128-B-line aligned; variant 70)
template <int K, int PD, int C, bool SC, int CP = 0, int KHO = 0>
__global__ __launch_bounds__(256) void k_diffuse_ps(const double *__restrict__ src, double *dst, int64_t field_stride,
                                                    int ny, int out_lo, int out_hi, int in_lo, int in_hi,
                                                    int top_reflect, int bot_reflect, int rows_per_chunk, int tiles_x,
                                                    int chunks_y, int n_fields, double coef, double c4, double cK,
                                                    const double *__restrict__ uniform, const VkPsCouple cp,
                                                    int gap_lo, int gap_hi, int chunks_a, int ea, int eb) {
    constexpr int KH = KHO > 0 ? KHO : (K + C - 1) / C * C;      // halo columns per side: >= K, whole lanes
    constexpr int W = 64 * C - 2 * KH;           // columns written per tile
    const int blk = vk_xcd_block<4>((int)blockIdx.x, (int)gridDim.x);
    const int wave = __builtin_amdgcn_readfirstlane((int)(blk * (blockDim.x >> 6) + (threadIdx.x >> 6)));
    const int lane = threadIdx.x & 63;
    if (wave >= tiles_x * chunks_y * n_fields) return;
    int tx, ty, f;
    vk_tile_of(wave, tiles_x, chunks_y, n_fields, ea, eb, tx, ty, f);
    // rows [gap_lo, gap_hi) are not written (two strips in one launch, vk_diffuse_part):
    // the first chunks_a chunks tile [out_lo, gap_lo), the rest [gap_hi, out_hi)
    const bool second = ty >= chunks_a;
    const int c0 = second ? gap_hi + (ty - chunks_a) * rows_per_chunk : out_lo + ty * rows_per_chunk;
    const int c1 = min(c0 + rows_per_chunk, second ? out_hi : gap_lo);
    const int x0 = tx * W;
    // agent coupling: the gather reads the plane before this pass changes anything
    if (cp.mode & 1) vk_couple_gather(cp, src + (int64_t)f * field_stride, f, ny, x0, W, c0, c1, lane);
    // a uniform plane keeps its values (zero delta); the exchange still applies
    if (!(uniform && uniform[2 * f] == uniform[2 * f + 1]))
        ps_plane<K, PD, C, SC, CP, KH, W>(src, dst, field_stride, ny, in_lo, in_hi, top_reflect, bot_reflect, coef,
                                          c4, cK, f, x0, c0, c1, lane);
    if (cp.mode & 2) vk_couple_exchange(cp, dst + (int64_t)f * field_stride, f, ny, x0, W, c0, c1, lane);
}

template <int K, int PD, int C, int CP = 0, int KHO = 0>
void launch(hipStream_t st, const double *src, double *dst, int nf, int64_t fs, int ny, int out_lo, int out_hi,
            int in_lo, int in_hi, int top, int bot, double coef, const double *mm, const VkPsCouple *cp,
            int gap_lo = -1, int gap_hi = -1) {
    constexpr int KH = KHO > 0 ? KHO : (K + C - 1) / C * C;
    constexpr int W = 64 * C - 2 * KH;
    const int tiles_x = (ny + W - 1) / W;
    if (!(gap_lo >= out_lo && gap_lo <= gap_hi && gap_hi <= out_hi)) gap_lo = gap_hi = out_hi;
    const int rows_a = gap_lo - out_lo, rows_b = out_hi - gap_hi;
    const int rch = chunk_rows(rows_a + rows_b, tiles_x, nf);
    const int chunks_a = (rows_a + rch - 1) / rch;
    const int chunks_y = chunks_a + (rows_b + rch - 1) / rch;
    const int waves = tiles_x * chunks_y * nf;
    int ea = 0, eb = 0;     // (two strips in one launch: only the side columns go first)
    if (chunks_a == chunks_y) vk_edge_chunks(K, out_lo, out_hi, rch, chunks_y, top, bot, ea, eb);
    const double c4 = 1.0 - 4.0 * coef;
    VkPsCouple none = {};
    const VkPsCouple &cpl = cp ? *cp : none;
    // the rescaled form while c4^-K stays far from overflow (|c4| >= 1e-3, i.e. coef
    // not within 2.5e-4 of 1/4); coef = 0 gives the identity exactly
    if (fabs(c4) >= 1e-3) {
        double cK = 1.0;
        for (int k = 0; k < K; ++k) cK *= c4;
        hipLaunchKernelGGL((k_diffuse_ps<K, PD, C, true, CP, KHO>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst, fs, ny,
                           out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef / c4, c4, cK, mm, cpl,
                           gap_lo, gap_hi, chunks_a, ea, eb);
    } else {
        hipLaunchKernelGGL((k_diffuse_ps<K, PD, C, false, CP, KHO>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst, fs,
                           ny, out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef, c4, 1.0, mm, cpl,
                           gap_lo, gap_hi, chunks_a, ea, eb);
    }
}

}  // namespace vk_ps

