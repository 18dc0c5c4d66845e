// Stage-split pair-sum passes (variant 40): the tolerance-mode pass of
// vk_stencil_ps.h with its K pipeline stages spread over the NW waves of a
// workgroup, so that one workgroup streams a TALL chunk of a column tile.
//
// Why.  A variant-20 wave carries all K stages of its tile in VGPRs (145 at
// K = 10, 3 waves per SIMD), so to keep enough waves in flight its chunks are
// short (34 rows), and every chunk re-reads and re-computes the 2K rows of its
// vertical halo: 54 rows read per 34 written (1.59x), 19 fill iterations per 34
// steady ones.  The counters say the pass moves 1.39x its algorithmic bytes at
// the copy rate (profiles/pmc_stencil_ps_d10_r34.json): its time is its traffic.
//
// Here wave s of a workgroup owns stages [s K / NW, (s+1) K / NW).  Every
// iteration each wave runs its stages on one row and hands the last stage's
// output row to wave s+1 through LDS (one 16-B write and read per lane), and the
// workgroup meets at one barrier.  Wave s therefore runs the single-wave
// pipeline of variant 20 with a lag of s iterations, on its share of the
// registers: a wave holds 2 of the 10 stages, so chunks can be ~4x taller at
// the same occupancy -- fewer halo rows read (R + 2K over R) and fewer fill
// iterations.  Wave 0 also loads the rows (the prefetch ring), wave NW-1 stores.
//
// Every cell goes through ps_stage with the same operands in the same order as
// in variant 20, so the two are bit-identical (tests/test_stencil_modes.py).
#pragma once

#include "vk_stencil_ps.h"

namespace vk_sp {

using vk_ps::clamp_row;
using vk_ps::dv2;
using vk_ps::PsArgs;
using vk_ps::PsLane;

template <int K, int NW, int S>
struct Stages {
    static constexpr int Q0 = S * K / NW;          // first stage of wave S
    static constexpr int Q1 = (S + 1) * K / NW;    // one past its last
    static constexpr int NS = Q1 - Q0;
};

template <int K, int PD, int C, int NS, bool RING>
struct SpState {
    static constexpr int NR = PD + 2;
    double ring[RING ? NR : 1][C];         // wave 0: stage 0's rows i-1, i and PD in flight
    double Wa[NS][C], Wb[NS][C];           // stage Q0 + l: centre / fresh rows, roles swap each iteration
    double Da[NS][C], Db[NS][C];           // its d rows, double-buffered the same way
};

// The LDS row a wave hands to the next: 64 lanes x C doubles, two slots per
// boundary (written at barrier step b into slot b & 1, read at step b + 1).
typedef __attribute__((address_space(3))) dv2 lds_dv2;

template <int C>
__device__ __forceinline__ void xfer_write(__attribute__((address_space(3))) double *slot, const double (&v)[C],
                                           int lane) {
#pragma unroll
    for (int j = 0; j < C; j += 2) {
        dv2 w;
        w.x = v[j];
        w.y = v[j + 1];
        *(lds_dv2 *)(slot + lane * C + j) = w;
    }
}

template <int C>
__device__ __forceinline__ void xfer_read(double (&v)[C], const __attribute__((address_space(3))) double *slot,
                                          int lane) {
#pragma unroll
    for (int j = 0; j < C; j += 2) {
        const dv2 w = *(const lds_dv2 *)(slot + lane * C + j);
        v[j] = w.x;
        v[j + 1] = w.y;
    }
}

typedef __attribute__((address_space(3))) double lds_double;

struct SpXfer {
    lds_double *in;      // boundary (S-1 -> S): slots of 64 * C doubles (unused by wave 0)
    lds_double *out;     // boundary (S -> S+1) (unused by the last wave)
    int lane;
};

// The workgroup barrier of one iteration.  Only LDS is ordered: the hand-off row
// written before it is read after it.  Wave 0's row prefetch and the last wave's
// stores stay in flight across it (a __syncthreads() fence would wait for them).
__device__ __forceinline__ void sp_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Local iteration i (ring phase U: row i sits in wave 0's ring slot U) of wave S:
// stages [Q0, min(Q1, ACT)) on one row each, then the hand-off and the barrier.
template <int K, int PD, int C, int NW, int S, bool GL, bool GR, bool EY, bool SC, int CP, int ACT, bool STORE, int U>
__device__ __forceinline__ void sp_iter(SpState<K, PD, C, Stages<K, NW, S>::NS, S == 0> &St, const PsArgs &A,
                                        const PsLane &L, SpXfer &X, int i) {
    using St_ = Stages<K, NW, S>;
    constexpr int Q0 = St_::Q0, Q1 = St_::Q1;
    constexpr int NR = PD + 2;
    constexpr int P = U & 1;
    __builtin_amdgcn_sched_barrier(0);
    double r0c[C], r0f[C];
    if constexpr (S == 0) {
        vk_ps::ps_load<C, GL && GR && EY, CP & 1>(St.ring[(U + PD) % NR],
                                                   A.s + clamp_row(i + PD, A.in_lo, A.in_hi) * L.ny64, L);
#pragma unroll
        for (int j = 0; j < C; ++j) {
            r0c[j] = St.ring[(U + NR - 1) % NR][j];
            r0f[j] = St.ring[U][j];
        }
    } else {
        // stage Q0 - 1's output of this local iteration, handed over one barrier
        // step ago (local iteration i of wave S-1 ran at step i + S - 1)
        double(&fr)[C] = P == 0 ? St.Wb[0] : St.Wa[0];
        xfer_read<C>(fr, X.in + ((U + S + 1) & 1) * 64 * C, X.lane);
    }
#pragma unroll
    for (int q = Q0; q < (Q1 < ACT ? Q1 : ACT); ++q) {
        const int l = q - Q0;
        const int r = i - 1 - q;
        const double(&cn)[C] = q == 0 ? r0c : (P == 0 ? St.Wa[l] : St.Wb[l]);
        const double(&fr)[C] = q == 0 ? r0f : (P == 0 ? St.Wb[l] : St.Wa[l]);
        const double(&dold)[C] = P == 0 ? St.Da[l] : St.Db[l];
        double(&dnew)[C] = P == 0 ? St.Db[l] : St.Da[l];
        double v[C];
        vk_ps::ps_stage<C, GL, GR, EY, SC>(cn, fr, dold, dnew, v, EY && r == A.top, EY && r == A.bot, q == 0, L,
                                           A.coef, A.c4);
        if (q + 1 < Q1) {
            double(&nx)[C] = P == 0 ? St.Wb[l + 1] : St.Wa[l + 1];
#pragma unroll
            for (int j = 0; j < C; ++j) nx[j] = v[j];
        } else if (q + 1 < K) {
            xfer_write<C>(X.out + ((U + S) & 1) * 64 * C, v, X.lane);
        } else if (STORE) {
            if (SC) {
#pragma unroll
                for (int j = 0; j < C; ++j) v[j] *= A.cK;
            }
            vk_ps::ps_store<C, GL && GR && EY, CP & 2>(A.d + (int64_t)(i - K) * L.ny64, v, L);
        }
    }
    sp_sync();
}

template <int K, int PD, int C, int NW, int S, bool GL, bool GR, bool EY, bool SC, int CP, int T>
__device__ __forceinline__ void sp_fill(SpState<K, PD, C, Stages<K, NW, S>::NS, S == 0> &St, const PsArgs &A,
                                        const PsLane &L, SpXfer &X, int is) {
    if constexpr (T < 2 * K - 1) {
        constexpr int ACT = T / 2 + 1 < K ? T / 2 + 1 : K;
        sp_iter<K, PD, C, NW, S, GL, GR, EY, SC, CP, ACT, false, T % (PD + 2)>(St, A, L, X, is + T);
        sp_fill<K, PD, C, NW, S, GL, GR, EY, SC, CP, T + 1>(St, A, L, X, is);
    }
}

template <int K, int PD, int C, int NW, int S, bool GL, bool GR, bool EY, bool SC, int CP, int PH, int u>
__device__ __forceinline__ void sp_tail(SpState<K, PD, C, Stages<K, NW, S>::NS, S == 0> &St, const PsArgs &A,
                                        const PsLane &L, SpXfer &X, int i, int n) {
    constexpr int NR = PD + 2;
    if constexpr (u < NR - 1) {
        if (u < n) {
            sp_iter<K, PD, C, NW, S, GL, GR, EY, SC, CP, K, true, (PH + u) % NR>(St, A, L, X, i + u);
            sp_tail<K, PD, C, NW, S, GL, GR, EY, SC, CP, PH, u + 1>(St, A, L, X, i, n);
        }
    }
}

template <int K, int PD, int C, int NW, int S, bool GL, bool GR, bool EY, bool SC, int CP, int... Us>
__device__ __forceinline__ void sp_steady(std::integer_sequence<int, Us...>,
                                          SpState<K, PD, C, Stages<K, NW, S>::NS, S == 0> &St, const PsArgs &A,
                                          const PsLane &L, SpXfer &X, int i, int i1) {
    constexpr int NR = PD + 2;
    constexpr int PH = (2 * K - 1) % NR;
    for (; i + NR <= i1; i += NR) (sp_iter<K, PD, C, NW, S, GL, GR, EY, SC, CP, K, true, (PH + Us) % NR>(St, A, L, X, i + Us), ...);
    sp_tail<K, PD, C, NW, S, GL, GR, EY, SC, CP, PH, 0>(St, A, L, X, i, i1 - i);
}

// One wave's program for the workgroup's chunk: S idle barrier steps (the lag),
// the single-wave pipeline on its stages, NW-1-S idle steps -- every wave meets
// the same 2K-1 + (c1-c0) + NW-1 barriers.
template <int K, int PD, int C, int NW, int S, bool GL, bool GR, bool EY, bool SC, int CP>
__device__ __forceinline__ void sp_body(const PsArgs &A, const PsLane &L, SpXfer &X, int c0, int c1) {
    constexpr int NR = PD + 2;
    using St_ = Stages<K, NW, S>;
    SpState<K, PD, C, St_::NS, S == 0> St;
#pragma unroll
    for (int l = 0; l < St_::NS; ++l)
#pragma unroll
        for (int j = 0; j < C; ++j) St.Wa[l][j] = St.Wb[l][j] = St.Da[l][j] = St.Db[l][j] = 0.0;
    const int is = c0 - K + 1;
    if constexpr (S == 0) {
        vk_ps::ps_load<C, GL && GR && EY, CP & 1>(St.ring[NR - 1], A.s + clamp_row(is - 1, A.in_lo, A.in_hi) * L.ny64, L);
#pragma unroll
        for (int u = 0; u < PD; ++u)
            vk_ps::ps_load<C, GL && GR && EY, CP & 1>(St.ring[u], A.s + clamp_row(is + u, A.in_lo, A.in_hi) * L.ny64, L);
    }
    for (int b = 0; b < S; ++b) sp_sync();
    sp_fill<K, PD, C, NW, S, GL, GR, EY, SC, CP, 0>(St, A, L, X, is);
    sp_steady<K, PD, C, NW, S, GL, GR, EY, SC, CP>(std::make_integer_sequence<int, NR>(), St, A, L, X, c0 + K, c1 + K);
    for (int b = S + 1; b < NW; ++b) sp_sync();
}

// body: 0 interior, 1 side tile (a plane side in reach, no reflected row: 16-B
// accesses and both ghost fixes, as vk_stencil_ps.h's side body), 2 general
template <int K, int PD, int C, int NW, bool SC, int CP, int S = 0>
__device__ __forceinline__ void sp_dispatch(int w, int body, const PsArgs &A, const PsLane &L, SpXfer &X,
                                            int c0, int c1) {
    if constexpr (S < NW) {
        if (w == S) {
            if (body == 2 || !SC)
                sp_body<K, PD, C, NW, S, true, true, true, SC, CP>(A, L, X, c0, c1);
            else if constexpr (SC) {
                if (body == 1)
                    sp_body<K, PD, C, NW, S, true, true, false, SC, CP>(A, L, X, c0, c1);
                else
                    sp_body<K, PD, C, NW, S, false, false, false, SC, CP>(A, L, X, c0, c1);
            }
        } else {
            sp_dispatch<K, PD, C, NW, SC, CP, S + 1>(w, body, A, L, X, c0, c1);
        }
    }
}

// One workgroup = one (column tile, chunk of output rows, plane).  The tile
// mapping is the plane's: tile tx of chunk ty, chunks in row order.
template <int K, int PD, int C, int NW, bool SC, int CP = 0>
__global__ __launch_bounds__(64 * NW) void k_diffuse_sp(const double *__restrict__ src, double *dst,
                                                       int64_t field_stride, int ny, int out_lo, int out_hi, int in_lo,
                                                       int in_hi, int top_reflect, int bot_reflect, int rows_per_chunk,
                                                       int tiles_x, int chunks_y, int nf, int ea, int eb, double coef,
                                                       double c4, double cK, const double *__restrict__ uniform) {
    constexpr int KH = (K + C - 1) / C * C;
    constexpr int W = 64 * C - 2 * KH;
    constexpr int SLOTS = 2;     // hand-off slots per boundary
    __shared__ __attribute__((aligned(16))) double xfer[(NW > 1 ? NW - 1 : 1) * SLOTS * 64 * C];
    const int wg = blockIdx.x;
    const int w = __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int lane = threadIdx.x & 63;
    int tx, ty, f;
    vk_tile_of(wg, tiles_x, chunks_y, nf, ea, eb, tx, ty, f);   // edge tiles first (vk_stencil_kernels.h)
    if (uniform && uniform[2 * f] == uniform[2 * f + 1]) return;     // a uniform plane keeps its values
    const int c0 = out_lo + ty * rows_per_chunk;
    const int c1 = min(c0 + rows_per_chunk, out_hi);
    const int x0 = tx * W;
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
    SpXfer X;
    lds_double *xl = (lds_double *)xfer;
    X.in = xl + (w > 0 ? w - 1 : 0) * SLOTS * 64 * C;
    X.out = xl + (w < NW - 1 ? w : 0) * SLOTS * 64 * C;
    X.lane = lane;
    const bool gl = x0 - KH <= 0;
    const bool gr = x0 - KH + 64 * C >= ny;
    const bool ey = (top_reflect >= c0 - 2 * K - 2 && top_reflect <= c1 + 2 * K) ||
                    (bot_reflect >= c0 - 2 * K - 2 && bot_reflect <= c1 + 2 * K);
    const int body = (ey || (gl && gr) || (ny % C) != 0) ? 2 : ((gl || gr) ? 1 : 0);
    sp_dispatch<K, PD, C, NW, SC, CP>(w, body, A, L, X, c0, c1);
}

// Workgroups of the kernel resident on the device at once (occupancy x CUs; 5 x 256
// on MI355X at 65 VGPRs), asked once per process.
template <int K, int PD, int C, int NW, int CP>
int resident_groups() {
    static int cached = 0;
    if (cached == 0) {
        int dev = 0, cus = 0, per_cu = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, k_diffuse_sp<K, PD, C, NW, true, CP>, 64 * NW, 0) !=
                hipSuccess)
            return 1280;
        cached = per_cu * cus > 0 ? per_cu * cus : 1280;
    }
    return cached;
}

// Auto chunk rows: whole rounds of resident workgroups.  One round holds
// per_round = resident / (tile columns x planes) chunks; the pass takes k rounds,
// k chosen so that chunks stay near 75 rows (taller chunks re-read less halo, but
// one round of very tall chunks leaves each SIMD's waves exposed).  Measured
// (profiles/r05/r05p-r05r, ms per 100 substeps): C3's 1024^2 x 2 at 16 rows
// (one round) 0.222 ms per step against 0.286 / 0.258 at 8 / 20 rows and 0.320 for
// the 9-deep variant-20 plan; a middle rank's band at N = 8 / 4 / 2 at 45 / 77 / 68
// rows 0.333 / 0.498 / 0.803 ms against 0.339 / 0.511 / 0.803 with the fixed rows.
inline int round_rows(int out_rows, int per_round) {
    per_round = per_round > 0 ? per_round : 1;
    const int rows1 = (out_rows + per_round - 1) / per_round;
    int k = (int)(rows1 / 75.0 + 0.5);
    k = k > 0 ? k : 1;
    const int rows = (out_rows + per_round * k - 1) / (per_round * k);
    return rows > 8 ? rows : 8;
}

template <int K, int PD, int C, int NW, int CP = 0>
void launch(hipStream_t st, const double *src, double *dst, int nf, int64_t fs, int ny, int out_lo, int out_hi,
            int in_lo, int in_hi, int top, int bot, double coef, const double *mm, int rows) {
    constexpr int KH = (K + C - 1) / C * C;
    constexpr int W = 64 * C - 2 * KH;
    const int tiles_x = (ny + W - 1) / W;
    if (rows <= 0) rows = round_rows(out_hi - out_lo, resident_groups<K, PD, C, NW, CP>() / (tiles_x * nf));
    const int chunks_y = (out_hi - out_lo + rows - 1) / rows;
    const int groups = tiles_x * chunks_y * nf;
    int ea = 0, eb = 0;
    vk_edge_chunks(K, out_lo, out_hi, rows, chunks_y, top, bot, ea, eb);
    const double c4 = 1.0 - 4.0 * coef;
    if (fabs(c4) >= 1e-3) {
        double cK = 1.0;
        for (int k = 0; k < K; ++k) cK *= c4;
        hipLaunchKernelGGL((k_diffuse_sp<K, PD, C, NW, true, CP>), dim3(groups), dim3(64 * NW), 0, st, src, dst, fs,
                           ny, out_lo, out_hi, in_lo, in_hi, top, bot, rows, tiles_x, chunks_y, nf, ea, eb, coef / c4, c4, cK,
                           mm);
    } else {
        hipLaunchKernelGGL((k_diffuse_sp<K, PD, C, NW, false, CP>), dim3(groups), dim3(64 * NW), 0, st, src, dst, fs,
                           ny, out_lo, out_hi, in_lo, in_hi, top, bot, rows, tiles_x, chunks_y, nf, ea, eb, coef, c4, 1.0,
                           mm);
    }
}

}  // namespace vk_sp
