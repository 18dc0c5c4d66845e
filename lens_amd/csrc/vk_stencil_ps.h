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

__device__ __forceinline__ __amdgpu_buffer_rsrc_t row_rsrc(const double *row, int ny, bool live = true) {
    // same descriptor word 3 as the variant-13 buffer stores of round 3; a row
    // that is not live gets 0 records: its loads return zeros and touch no memory
    return __builtin_amdgcn_make_buffer_rsrc((void *)row, 0, live ? ny * 8 : 0, 0x00020000);
}

// CL = the general edge body (a row width the 16-B accesses cannot tile, a plane
// one tile wide, or a reflected row in reach): columns clamped per element and
// stores masked per column.  Otherwise 16-B buffer accesses: a lane left or
// right of the plane loads zeros (its columns are halo) and stores nothing.
// CP: bit 0 = streaming (nt) loads (A/B only), bit 1 = plain (cached) stores -- the 10-deep
// pass's choice when its planes fit the MALL (vk_stencil_ps10.hip); 0 = plain loads and
// streaming stores, the default
template <int C, bool CL, int CP = 0>
__device__ __forceinline__ void ps_load(double (&out)[C], const double *__restrict__ row, const PsLane &L,
                                        bool live = true) {
    if constexpr (!CL) {
        const __amdgpu_buffer_rsrc_t rs = row_rsrc(row, L.ny, live);
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
    int row_end;            // the chunk's last input row + 1 (c1 + K): the ring's lookahead past it is not loaded
    double coef, c4, cK;
};

__device__ __forceinline__ int64_t clamp_row(int r, int lo, int hi) { return (int64_t)min(max(r, lo), hi - 1); }

// Vertical stash (VS > 0, variants 60-62): a workgroup's 4 waves take 4 vertically
// adjacent chunks of one column tile.  Chunk w's last 2K input rows are chunk w+1's
// first 2K: the lower wave has them in registers during its fill, so it writes the
// last VS of them to LDS, and the upper wave reads them from there ~60 iterations
// later instead of from HBM (no cache bridges that distance: the rows are evicted
// long before, profiles/r03/r03u/).  A flag per boundary, set after the rows (LDS
// executes one wave's operations in order), orders the two waves.  The top wave
// writes its rows to a trash row (no branch in the fill: a branch there costs 13
// VGPRs), and the reads sit in an end segment unrolled at compile time (a branch per
// iteration costs 33).
typedef __attribute__((address_space(3))) i4v lds_i4v;
typedef __attribute__((address_space(3))) volatile int lds_flag;
struct PsStash {
    lds_i4v *wr;        // the rows this wave hands to the wave above (the trash row for wave 0)
    int wstride;        // i4v elements between written rows (0: the trash row)
    lds_flag *wflag;
    const lds_i4v *rd;  // the rows handed up by the wave below (the zero row if not linked)
    int rstride;        // i4v elements between read rows (0: the zero row)
    lds_flag *rflag;    // (a flag that is set if not linked)
    bool linked;        // the chunk below is this group's: it hands its rows up
    int lane;
};

__device__ __forceinline__ void stash_wait(const PsStash &X) {
    while (*X.rflag == 0) __builtin_amdgcn_s_sleep(1);
    // the rows were written before the flag: nothing may be read ahead of it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
}

// Iteration i at ring phase U (row i sits in ring slot U): prefetch row i+PD,
// run stages [0, ACT), store row i-K if STORE.  FT >= 0: fill iteration FT (the
// stash rows are written there).  SRC: where row i+PD comes from -- 0 HBM (not
// loaded past the chunk's cone), 1 the stash (slot SLOT), 2 nowhere (past the cone).
template <int K, int PD, int C, bool GL, bool GR, bool EY, bool SC, int CP, int VS, int ACT, bool STORE, int U,
          int FT = -1, int SRC = 0, int SLOT = 0>
__device__ __forceinline__ void ps_iter(PsState<K, PD, C> &S, const PsArgs &A, const PsLane &L, const PsStash &X,
                                        int i) {
    constexpr int NR = PD + 2;
    constexpr int P = U & 1;
    // keep iterations in program order: the scheduler would otherwise hoist the
    // unrolled group's row loads (and their registers) to its top
    __builtin_amdgcn_sched_barrier(0);
    double r0c[C], r0f[C];                 // stage 0's rows i-1 and i
    const int row = i + PD;
    double(&slot)[C] = S.ring[(U + PD) % NR];
    if constexpr (SRC == 0) {
        // the last PD iterations' lookahead rows lie past the chunk's cone (4 of 88 rows read per
        // 64-row chunk): not loaded
        ps_load<C, GL && GR && EY, CP>(slot, A.s + clamp_row(row, A.in_lo, A.in_hi) * L.ny64, L, row < A.row_end);
    } else if constexpr (SRC == 1) {
        // a linked chunk reads the stash (its HBM load has 0 records: zeros, no traffic);
        // any other reads the zero row and loads from HBM; the two are OR-ed
        static_assert(C == 2, "the stash holds one 16-B element per lane and row");
        double g[C];
        ps_load<C, GL && GR && EY, CP>(g, A.s + clamp_row(row, A.in_lo, A.in_hi) * L.ny64, L, !X.linked);
        if constexpr (SLOT == 0) stash_wait(X);
        const i4v y = X.rd[SLOT * X.rstride + X.lane];
        const i4v z = __builtin_bit_cast(i4v, make_double2(g[0], g[1])) | y;
        const double2 v = __builtin_bit_cast(double2, z);
        slot[0] = v.x;
        slot[1] = v.y;
    }
#pragma unroll
    for (int j = 0; j < C; ++j) {
        r0c[j] = S.ring[(U + NR - 1) % NR][j];
        r0f[j] = S.ring[U][j];
    }
    if constexpr (VS > 0 && FT >= 0 && FT + 1 >= 2 * K - VS) {
        // r0f is this chunk's input row FT + 1 (counted from c0 - K)
        X.wr[(FT + 1 - (2 * K - VS)) * X.wstride + X.lane] = __builtin_bit_cast(i4v, make_double2(r0f[0], r0f[1]));
        if constexpr (FT == 2 * K - 2) {
            asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
            *X.wflag = 1;
        }
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

template <int K, int PD, int C, bool GL, bool GR, bool EY, bool SC, int CP, int VS, int T>
__device__ __forceinline__ void ps_fill(PsState<K, PD, C> &S, const PsArgs &A, const PsLane &L, const PsStash &X, int is) {
    if constexpr (T < 2 * K - 1) {
        constexpr int ACT = T / 2 + 1 < K ? T / 2 + 1 : K;
        ps_iter<K, PD, C, GL, GR, EY, SC, CP, VS, ACT, false, T % (PD + 2), T>(S, A, L, X, is + T);
        ps_fill<K, PD, C, GL, GR, EY, SC, CP, VS, T + 1>(S, A, L, X, is);
    }
}

// The last (i1 - i) < NR iterations, nested (iteration u runs only if u-1 ran),
// so that no state has to be merged across a skipped iteration: a flat list of
// guarded iterations keeps both versions of every row live and costs ~60 VGPRs.
template <int K, int PD, int C, bool GL, bool GR, bool EY, bool SC, int CP, int VS, int PH, int u>
__device__ __forceinline__ void ps_tail(PsState<K, PD, C> &S, const PsArgs &A, const PsLane &L, const PsStash &X, int i,
                                        int n) {
    constexpr int NR = PD + 2;
    if constexpr (u < NR - 1) {
        if (u < n) {
            ps_iter<K, PD, C, GL, GR, EY, SC, CP, VS, K, true, (PH + u) % NR>(S, A, L, X, i + u);
            ps_tail<K, PD, C, GL, GR, EY, SC, CP, VS, PH, u + 1>(S, A, L, X, i, n);
        }
    }
}

template <int K, int PD, int C, bool GL, bool GR, bool EY, bool SC, int CP, int VS, int... Us>
__device__ __forceinline__ void ps_steady(std::integer_sequence<int, Us...>, PsState<K, PD, C> &S, const PsArgs &A,
                                          const PsLane &L, const PsStash &X, int i, int i1) {
    constexpr int NR = PD + 2;
    constexpr int PH = (2 * K - 1) % NR;    // ring phase of the first steady iteration
    for (; i + NR <= i1; i += NR)
        (ps_iter<K, PD, C, GL, GR, EY, SC, CP, VS, K, true, (PH + Us) % NR>(S, A, L, X, i + Us), ...);
    ps_tail<K, PD, C, GL, GR, EY, SC, CP, VS, PH, 0>(S, A, L, X, i, i1 - i);
}

// A linked chunk (VS > 0) is VS_RCH rows tall: after NG groups of NR iterations from
// HBM, its last iterations are unrolled with each row's source fixed at compile time.
constexpr int VS_RCH = 64;

template <int K, int PD, int C, bool GL, bool GR, bool EY, bool SC, int CP, int VS, int PH, int... Us>
__device__ __forceinline__ void ps_group(std::integer_sequence<int, Us...>, PsState<K, PD, C> &S, const PsArgs &A,
                                         const PsLane &L, const PsStash &X, int i) {
    constexpr int NR = PD + 2;
    (ps_iter<K, PD, C, GL, GR, EY, SC, CP, VS, K, true, (PH + Us) % NR>(S, A, L, X, i + Us), ...);
}

// iteration t (counted from c0 + K) of a linked chunk, t = T .. VS_RCH - 1
template <int K, int PD, int C, bool GL, bool GR, bool EY, bool SC, int CP, int VS, int PH, int T>
__device__ __forceinline__ void ps_end(PsState<K, PD, C> &S, const PsArgs &A, const PsLane &L, const PsStash &X,
                                       int i) {
    if constexpr (T < VS_RCH) {
        constexpr int NR = PD + 2;
        constexpr int TG = VS_RCH - VS - PD;            // rows t + PD < VS_RCH + K - VS come from HBM
        constexpr int SRC = T < TG ? 0 : (T < TG + VS ? 1 : 2);
        ps_iter<K, PD, C, GL, GR, EY, SC, CP, VS, K, true, (PH + T) % NR, -1, SRC, SRC == 1 ? T - TG : 0>(S, A, L, X,
                                                                                                          i);
        ps_end<K, PD, C, GL, GR, EY, SC, CP, VS, PH, T + 1>(S, A, L, X, i + 1);
    }
}

template <int K, int PD, int C, bool GL, bool GR, bool EY, bool SC, int CP, int VS>
__device__ __forceinline__ void ps_body(const PsArgs &A, const PsLane &L, const PsStash &X, int c0, int c1) {
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
    ps_fill<K, PD, C, GL, GR, EY, SC, CP, VS, 0>(S, A, L, X, is);
    // steady: i = c0+K .. c1+K-1, one stored row each (rows c0 .. c1-1)
    if constexpr (VS > 0) {
        // every chunk is VS_RCH rows (the launcher's condition): the source of every row is
        // known at compile time; no branch on `linked` (one after the fill costs ~100 VGPRs)
        constexpr int PH = (2 * K - 1) % NR;
        constexpr int NG = (VS_RCH - VS - PD) / NR;     // whole groups before the first stash row
        int i = c0 + K;
        for (int g = 0; g < NG; ++g, i += NR)
            ps_group<K, PD, C, GL, GR, EY, SC, CP, VS, PH>(std::make_integer_sequence<int, NR>(), S, A, L, X, i);
        ps_end<K, PD, C, GL, GR, EY, SC, CP, VS, PH, NG * NR>(S, A, L, X, i);
    } else {
        ps_steady<K, PD, C, GL, GR, EY, SC, CP, VS>(std::make_integer_sequence<int, NR>(), S, A, L, X, c0 + K, c1 + K);
    }
}

// The stencil work of one wave: its tile of plane f, output rows [c0, c1)
template <int K, int PD, int C, bool SC, int CP, int KH, int W, int VS = 0>
__device__ __forceinline__ void ps_plane(const double *__restrict__ src, double *dst, int64_t field_stride, int ny,
                                         int in_lo, int in_hi, int top_reflect, int bot_reflect, double coef,
                                         double c4, double cK, int f, int x0, int c0, int c1, int lane, PsStash &X) {
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
    A.row_end = c1 + K;
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
        ps_body<K, PD, C, true, true, true, SC, CP, VS>(A, L, X, c0, c1);
    else if constexpr (SC) {
        if (gl || gr)
            ps_body<K, PD, C, true, true, false, SC, CP, VS>(A, L, X, c0, c1);
        else
            ps_body<K, PD, C, false, false, false, SC, CP, VS>(A, L, X, c0, c1);
    }
}

template <int K, int PD, int C, bool SC, int CP = 0>
__global__ __launch_bounds__(256) void k_diffuse_ps(const double *__restrict__ src, double *dst, int64_t field_stride,
                                                    int ny, int out_lo, int out_hi, int in_lo, int in_hi,
                                                    int top_reflect, int bot_reflect, int rows_per_chunk, int tiles_x,
                                                    int chunks_y, int n_fields, double coef, double c4, double cK,
                                                    const double *__restrict__ uniform, const VkPsCouple cp,
                                                    int gap_lo, int gap_hi, int chunks_a, int ea, int eb) {
    constexpr int KH = (K + C - 1) / C * C;      // halo columns per side: >= K, whole lanes
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
    if (!(uniform && uniform[2 * f] == uniform[2 * f + 1])) {
        PsStash X = {};
        ps_plane<K, PD, C, SC, CP, KH, W>(src, dst, field_stride, ny, in_lo, in_hi, top_reflect, bot_reflect, coef,
                                          c4, cK, f, x0, c0, c1, lane, X);
    }
    if (cp.mode & 2) vk_couple_exchange(cp, dst + (int64_t)f * field_stride, f, ny, x0, W, c0, c1, lane);
}

// Variant 60: the pass with the vertical stash (PsStash above).  Block = group g of
// 4 chunks (ty = 4g + w) of one column tile; groups in the edge-first, XCD-windowed
// order of the wave tiles (a group is an edge group if any of its chunks is).
// GEO (A/B of what the stash costs): 0 = the stash; 1 = the same groups, no row read
// from the stash; 2 = variant 20's tile order (4 side-by-side tiles per block), no stash
template <int K, int PD, int C, bool SC, int VS, int XM, int GEO = 0>
__global__ __launch_bounds__(256) void k_diffuse_ps_vs(const double *__restrict__ src, double *dst,
                                                       int64_t field_stride, int ny, int out_lo, int out_hi, int in_lo,
                                                       int in_hi, int top_reflect, int bot_reflect, int rows_per_chunk,
                                                       int tiles_x, int chunks_y, int groups_y, int n_fields,
                                                       double coef, double c4, double cK,
                                                       const double *__restrict__ uniform, const VkPsCouple cp, int ga,
                                                       int gb) {
    constexpr int KH = (K + C - 1) / C * C;
    constexpr int W = 64 * C - 2 * KH;
    // three boundaries' rows, the trash row (wave 0's writes), the zero row
    __shared__ i4v stash[(3 * VS + 2) * 64];
    __shared__ int flags[5];
    const int blk = vk_xcd_block<XM>((int)blockIdx.x, (int)gridDim.x);
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    // flag w: wave w+1 has written its rows for wave w.  Every wave passes the one
    // barrier below before any flag is set or read.
    if (lane == 0) flags[w] = 0;
    if (w == 0) {
        stash[(3 * VS + 1) * 64 + lane] = i4v{0, 0, 0, 0};
        if (lane == 0) flags[4] = 1;
    }
    __syncthreads();
    int tx, ty, f;
    if constexpr (GEO == 2) {
        const int wave = blk * 4 + w;
        if (wave >= tiles_x * chunks_y * n_fields) return;
        vk_tile_of(wave, tiles_x, chunks_y, n_fields, ga, gb, tx, ty, f);
    } else {
        if (blk >= tiles_x * groups_y * n_fields) return;
        int g;
        vk_tile_of(blk, tiles_x, groups_y, n_fields, ga, gb, tx, g, f);
        ty = 4 * g + w;
        if (ty >= chunks_y) return;
    }
    const int c0 = out_lo + ty * rows_per_chunk;
    const int c1 = min(c0 + rows_per_chunk, out_hi);
    const int x0 = tx * W;
    if (cp.mode & 1) vk_couple_gather(cp, src + (int64_t)f * field_stride, f, ny, x0, W, c0, c1, lane);
    if (!(uniform && uniform[2 * f] == uniform[2 * f + 1])) {
        PsStash X;
        X.lane = lane;
        // wave 0 has no wave above: its rows go to the trash row after the three areas
        X.wr = (lds_i4v *)&stash[(w > 0 ? (w - 1) * VS : 3 * VS) * 64];
        X.wstride = w > 0 ? 64 : 0;
        X.wflag = (lds_flag *)&flags[w > 0 ? w - 1 : 3];
        // the chunk below is this group's (every chunk is VS_RCH rows: launch_vs)
        X.linked = GEO == 0 && w < 3 && ty + 1 < chunks_y;
        X.rd = (const lds_i4v *)&stash[(X.linked ? w * VS : 3 * VS + 1) * 64];
        X.rstride = X.linked ? 64 : 0;
        X.rflag = (lds_flag *)&flags[X.linked ? w : 4];
        ps_plane<K, PD, C, SC, 0, KH, W, VS>(src, dst, field_stride, ny, in_lo, in_hi, top_reflect, bot_reflect,
                                             coef, c4, cK, f, x0, c0, c1, lane, X);
    }
    if (cp.mode & 2) vk_couple_exchange(cp, dst + (int64_t)f * field_stride, f, ny, x0, W, c0, c1, lane);
}

template <int K, int PD, int C, int CP = 0>
void launch(hipStream_t st, const double *src, double *dst, int nf, int64_t fs, int ny, int out_lo, int out_hi,
            int in_lo, int in_hi, int top, int bot, double coef, const double *mm, const VkPsCouple *cp,
            int gap_lo = -1, int gap_hi = -1) {
    constexpr int KH = (K + C - 1) / C * C;
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
        hipLaunchKernelGGL((k_diffuse_ps<K, PD, C, true, CP>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst, fs, ny,
                           out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef / c4, c4, cK, mm, cpl,
                           gap_lo, gap_hi, chunks_a, ea, eb);
    } else {
        hipLaunchKernelGGL((k_diffuse_ps<K, PD, C, false, CP>), dim3((waves + 3) / 4), dim3(256), 0, st, src, dst, fs,
                           ny, out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, nf, coef, c4, 1.0, mm, cpl,
                           gap_lo, gap_hi, chunks_a, ea, eb);
    }
}

template <int K, int PD, int C, int VS, int XM = 4, int GEO = 0>
bool launch_vs(hipStream_t st, const double *src, double *dst, int nf, int64_t fs, int ny, int out_lo, int out_hi,
               int in_lo, int in_hi, int top, int bot, double coef, const double *mm, const VkPsCouple *cp) {
    constexpr int KH = (K + C - 1) / C * C;
    constexpr int W = 64 * C - 2 * KH;
    const int tiles_x = (ny + W - 1) / W;
    const int rch = chunk_rows(out_hi - out_lo, tiles_x, nf);
    // every chunk exactly VS_RCH rows (the kernel's row plan is fixed at compile time)
    if (rch != VS_RCH || (out_hi - out_lo) % VS_RCH != 0) return false;
    const int chunks_y = (out_hi - out_lo + rch - 1) / rch;
    const int groups_y = (chunks_y + 3) / 4;
    int ea = 0, eb = 0;
    vk_edge_chunks(K, out_lo, out_hi, rch, chunks_y, top, bot, ea, eb);
    // groups holding an edge chunk go first, as the edge chunks do in the wave-tile order
    int ga = (ea + 3) / 4, gb = eb > 0 ? groups_y - (chunks_y - eb) / 4 : 0;
    if (ga + gb > groups_y) { ga = groups_y; gb = 0; }
    int blocks = tiles_x * groups_y * nf;
    if (GEO == 2) { ga = ea; gb = eb; blocks = (tiles_x * chunks_y * nf + 3) / 4; }
    const double c4 = 1.0 - 4.0 * coef;
    VkPsCouple none = {};
    const VkPsCouple &cpl = cp ? *cp : none;
    if (fabs(c4) >= 1e-3) {
        double cK = 1.0;
        for (int k = 0; k < K; ++k) cK *= c4;
        hipLaunchKernelGGL((k_diffuse_ps_vs<K, PD, C, true, VS, XM, GEO>), dim3(blocks), dim3(256), 0, st, src, dst, fs, ny,
                           out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, groups_y, nf, coef / c4, c4,
                           cK, mm, cpl, ga, gb);
    } else {
        hipLaunchKernelGGL((k_diffuse_ps_vs<K, PD, C, false, VS, XM, GEO>), dim3(blocks), dim3(256), 0, st, src, dst, fs, ny,
                           out_lo, out_hi, in_lo, in_hi, top, bot, rch, tiles_x, chunks_y, groups_y, nf, coef, c4, 1.0,
                           mm, cpl, ga, gb);
    }
    return true;
}

}  // namespace vk_ps

