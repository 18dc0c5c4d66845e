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
#include <vector>


#include "vk_internal.h"
#include "vk_stencil_launch.h"

constexpr int ST_BX = 256;  // columns per block (4 waves, 2 KiB per row load)
constexpr int ST_RB = 16;   // rows walked per block

// One substep over rows [lo, hi) of every plane.  Each lane walks down a
// column keeping up/centre/down in registers: one new row load, two shifted
// loads (left/right: L1 hits on the lines the wave just fetched), one store.
__global__ __launch_bounds__(ST_BX) void k_diffuse_substep(const double *__restrict__ src,
                                                           double *dst,
                                                           const double *f0,
                                                           int64_t field_stride, int ny, int lo, int hi,
                                                           int top_reflect, int bot_reflect, double coef,
                                                           const double *__restrict__ uniform, int delta_mode) {
    const int f = blockIdx.z;
    const int j = blockIdx.x * ST_BX + threadIdx.x;
    const int r0 = lo + blockIdx.y * ST_RB;
    if (j >= ny || r0 >= hi) return;
    const int r1 = min(r0 + ST_RB, hi);
    const double *s = src + (int64_t)f * field_stride;
    double *d = dst + (int64_t)f * field_stride;
    const double *g = f0 ? f0 + (int64_t)f * field_stride : nullptr;
    if (uniform && uniform[2 * f] == uniform[2 * f + 1]) {   // uniform plane: the delta is zero
        if (delta_mode)
            for (int r = r0; r < r1; ++r) d[(int64_t)r * ny + j] = 0.0;
        return;
    }
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
            // delta_mode: the reference's delta = field_new - field, applied
            // later by the accumulate updater (diffusion_field.py:394)
            const double base = g[(int64_t)r * ny + j];
            v = delta_mode ? v - base : base + (v - base);
        }
        d[(int64_t)r * ny + j] = v;
        up = c;
        c = down;
    }
}

int g_stencil_rows = 0;    // output rows per wave tile (vk_stencil_kernels.h chunk_rows); 0 = auto
// Exact mode: 2 / 3 = wave tile lag-1 prefetching 3 / 6 rows, 6 = variant 3 with
// streaming stores at depths 7 / 9 / 11 (the exact mode's kernel for every other
// setting).  Tolerance mode: 20 = pair-sum passes (vk_stencil_ps.h, the default; 2 /
// 3 / 6 select it too), 40 = the stage-split 10-deep pass (vk_stencil_sp.h; row
// bands), 70 = the 10-deep pair-sum pass with line-aligned tiles (96 written columns,
// vk_stencil_ps10.hip; the C4 default since round 6).  Tolerance-mode depths without a pair-sum pass (even depths below 10, 13,
// 15) run the exact wave tiles.
// Retired after A/B on the GPU: 0 (workgroup tile, LDS exchange),
// 1 (lag-2 wave tile), 4 (9 rows prefetched), 5 (4 waves/SIMD cap, spills),
// 7 (streaming loads), 8-11 (four columns per lane, compact boundary body, split
// stages, LDS-crossbar neighbours), 12-16 (prefetch ring, buffer stores, zigzag
// chunks, 6-row prefetch at depth 10), 21-32 (pair-sum prefetch depths, stagger,
// cache policies, one plane at a time, coupled-pass placements, the stage-0 ring as
// 16-B vectors: 30 tied variant 20 and was retired in round 5), the tolerance-mode
// FMA form of the wave tiles (4 FP64 ops per cell-substep; round 6) -- none faster.
static int g_stencil_kernel = 20;

extern "C" int vk_set_stencil_kernel(int32_t variant, int32_t rows) {
    const int prev = g_stencil_kernel;
    if (variant == 2 || variant == 3 || variant == 6 || variant == 20 || variant == 40 || variant == 70)
        g_stencil_kernel = variant;
    if (rows == 0 || (rows >= 8 && rows <= 4096)) g_stencil_rows = rows;
    return prev;
}

// 0 = bit-exact with scipy.ndimage.convolve (the default), 1 = tolerance mode: the
// pair-sum passes (3 FP64 ops per cell-substep instead of 6, vk_stencil_ps.h) and no
// base re-read in the final pass; fields agree with the exact mode to ~1e-14
// relative (tests/test_stencil_modes.py)
int g_stencil_mode = 0;

extern "C" int vk_set_stencil_mode(int32_t mode) {
    const int prev = g_stencil_mode;
    if (mode == 0 || mode == 1) g_stencil_mode = mode;
    return prev;
}

// max substeps per HBM pass: odd, 1 = one launch per substep; or 10, which plans a
// tolerance-mode whole step of a multiple of 10 substeps as 10-deep passes (three
// buffers: the field itself is free once the first pass has read it), other calls
// as depth 9
static int g_stencil_depth = 10;   // 10-deep block plan (odd-depth plan at 9 for other counts)

extern "C" int vk_set_stencil_depth(int32_t k) {
    const int prev = g_stencil_depth;
    if (k == 10) g_stencil_depth = 10;
    else if (k >= 1 && k <= 15) g_stencil_depth = k | 1;
    return prev;
}

// ---------------------------------------------------------------------------
// Segment timestamps (bench instrumentation inside a replayed HIP graph)
// ---------------------------------------------------------------------------

__global__ void k_timestamp(uint64_t *out, int idx) {
    if (threadIdx.x == 0) out[idx] = wall_clock64();
}

extern "C" int vk_timestamp(uint64_t *out, int32_t idx, vk_stream_t stream) {
    if (!out || idx < 0) {
        vk::set_error("vk_timestamp: bad arguments");
        return VK_ERR_ARG;
    }
    hipLaunchKernelGGL(k_timestamp, dim3(1), dim3(64), 0, (hipStream_t)stream, out, idx);
    return vk::launch_check("k_timestamp");
}

// The box's streaming-copy floor for a pass's planes: one 16-B element per thread,
// non-temporal store, one wave of workgroups over the whole buffer.  Of the copy
// shapes measured (scripts/micro/copy_floor.hip, profiles/r03/copy_floor.log) this
// one is fastest: 84.4 us for a 4096^2 x 2 FP64 pair, 6.36 TB/s; grid-stride copies
// and torch's copy_ reach 5.5-6.1.
typedef double vk_d2v __attribute__((ext_vector_type(2)));
__global__ __launch_bounds__(256) void k_copy_stream(const vk_d2v *__restrict__ s, vk_d2v *__restrict__ d, int64_t n) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i < n) __builtin_nontemporal_store(s[i], d + i);
}

extern "C" int vk_copy_stream(const double *src, double *dst, int64_t n_doubles, vk_stream_t stream) {
    if (!src || !dst || n_doubles < 0 || (n_doubles & 1) || (((uintptr_t)src | (uintptr_t)dst) & 15)) {
        vk::set_error("vk_copy_stream: bad arguments (16-B aligned buffers of an even number of doubles)");
        return VK_ERR_ARG;
    }
    const int64_t n = n_doubles / 2;
    if (n == 0) return VK_OK;
    hipLaunchKernelGGL(k_copy_stream, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       (const vk_d2v *)src, (vk_d2v *)dst, n);
    return vk::launch_check("k_copy_stream");
}

extern "C" int64_t vk_wall_clock_khz(void) {
    int dev = 0, khz = 0;
    if (hipGetDevice(&dev) != hipSuccess) return 0;
    if (hipDeviceGetAttribute(&khz, hipDeviceAttributeWallClockRate, dev) != hipSuccess) return 0;
    return khz;
}

// rows [lo, hi) of every non-uniform plane: dst <- src
__global__ __launch_bounds__(256) void k_copy_rows(const double *__restrict__ src, double *dst,
                                                   int64_t field_stride, int64_t off, int64_t count,
                                                   const double *__restrict__ uniform) {
    const int f = blockIdx.y;
    if (uniform && uniform[2 * f] == uniform[2 * f + 1]) return;
    const int64_t base = (int64_t)f * field_stride + off;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count; i += (int64_t)gridDim.x * blockDim.x)
        dst[base + i] = src[base + i];
}

// One fused pass of k >= 2 substeps, the kernel picked by mode / variant / depth;
// f0 != nullptr marks the exact mode's final pass (it re-reads the step-start plane).
// cp (nullable): the agent coupling the pass carries (vk_diffuse_coupled).
static void launch_pass(int k, hipStream_t s, const double *src, double *dst, const double *f0, int nf, int64_t fs,
                        int ny, int lo, int hi, int in_lo, int in_hi, int top, int bot, double coef, const double *mm,
                        const VkPsCouple *cp, bool strip = false) {
    if (g_stencil_mode == 1 && k <= 11 && ((k & 1) || k == 10)) {
        // tolerance mode, pair-sum passes (the final pass writes the new field as is);
        // they are instantiated for k = 3, 5, 7, 9, 10, 11 (an even k < 10 takes the
        // wave tiles below); variant 40: the stage-split 10-deep pass -- not for the
        // short edge strips of vk_diffuse_part (`strip`), whose passes are latency-bound
        // and run faster as single-wave tiles of a few rows
        if (g_stencil_kernel >= 40 && !strip &&
            vk_launch_sp(g_stencil_kernel, k, s, src, dst, f0, nf, fs, ny, lo, hi, in_lo, in_hi, top, bot, coef, mm, cp))
            return;
        if (k == 10 && g_stencil_kernel == 70 && !strip)
            vk_launch_ps10_aligned(k, s, src, dst, f0, nf, fs, ny, lo, hi, in_lo, in_hi, top, bot, coef, mm, cp);
        else if (k == 10) vk_launch_ps10(k, s, src, dst, f0, nf, fs, ny, lo, hi, in_lo, in_hi, top, bot, coef, mm, cp);
        else vk_launch_ps(k, s, src, dst, f0, nf, fs, ny, lo, hi, in_lo, in_hi, top, bot, coef, mm, cp);
    } else if (k == 10 || ((g_stencil_kernel == 6 || g_stencil_kernel >= 20) && (k == 7 || k == 9 || k == 11))) {
        // the exact mode's variant 6 (streaming stores), and its 10-deep whole-step plan
        vk_launch_wl6nt(k, s, src, dst, f0, nf, fs, ny, lo, hi, in_lo, in_hi, top, bot, coef, mm, cp);
    } else {
        // other depths (and variants 2 / 3): the plain-store wave tiles; the final pass
        // also streams the base plane (3 rows ahead), so it keeps the shallow row
        // prefetch and still fits 3 waves per SIMD
        auto launch = (g_stencil_kernel == 2 || f0) ? vk_launch_wl3 : vk_launch_wl6;
        launch(k, s, src, dst, f0, nf, fs, ny, lo, hi, in_lo, in_hi, top, bot, coef, mm, cp);
    }
}

// The odd-depth pass plan of a call's substeps [sub_begin, last]: the fewest odd
// depths <= the set depth that sum to the count (a sum of P odd numbers has the
// parity of P), as even as possible -- e.g. 100 = 8x9 + 4x7 rather than 11x9 + a
// lone single-substep pass.
static std::vector<int> odd_plan(int sub_count) {
    int depth = g_stencil_depth | 1;   // odd
    if (g_stencil_depth == 10) depth = 9;
    if (depth > 15) depth = 15;
    int passes = (sub_count + depth - 1) / depth;
    if ((passes & 1) != (sub_count & 1)) ++passes;
    std::vector<int> ks;
    for (int j = 0, left = passes; j < sub_count; --left) {
        const int rem = sub_count - j;   // rem has the parity of `left`
        int k = (rem + left - 1) / left;
        if ((k & 1) == 0) ++k;
        if (k > depth) k = depth;
        while (k > 1 && rem - k < left - 1) k -= 2;
        ks.push_back(k);
        j += k;
    }
    return ks;
}

static int diffuse_impl(double *field, double *work0, double *work1, int32_t n_fields, int64_t field_stride,
                        int32_t ny, int32_t row_lo, int32_t row_hi, int32_t lo_min, int32_t hi_max, int32_t edge_top,
                        int32_t edge_bot, int32_t sub_begin, int32_t sub_count, int32_t n_sub, double coeff_dt,
                        const double *uniform, int32_t part, int32_t split_m, vk_stream_t stream);

extern "C" int vk_diffuse(double *field, double *work0, double *work1, int32_t n_fields,
                          int64_t field_stride, int32_t ny, int32_t row_lo, int32_t row_hi, int32_t lo_min,
                          int32_t hi_max, int32_t edge_top, int32_t edge_bot, int32_t sub_begin,
                          int32_t sub_count, int32_t n_sub, double coeff_dt, const double *uniform,
                          vk_stream_t stream) {
    return diffuse_impl(field, work0, work1, n_fields, field_stride, ny, row_lo, row_hi, lo_min, hi_max, edge_top,
                        edge_bot, sub_begin, sub_count, n_sub, coeff_dt, uniform, VK_PART_ALL, 0, stream);
}

// Whether vk_diffuse_part can split this block: the 10-deep plan of a row band's
// block of 10 k substeps whose owned rows keep an interior through every pass.
static bool part_plan_ok(int32_t row_lo, int32_t row_hi, int32_t lo_min, int32_t hi_max, int32_t sub_count,
                         int32_t edge_top, int32_t edge_bot) {
    const bool halo_top = !edge_top && row_lo > lo_min, halo_bot = !edge_bot && row_hi < hi_max;
    return g_stencil_depth == 10 && sub_count % 10 == 0 && sub_count > 0 && (halo_top || halo_bot) &&
           row_hi - row_lo > 2 * sub_count;
}

extern "C" int vk_diffuse_part(double *field, double *work0, double *work1, int32_t n_fields, int64_t field_stride,
                               int32_t ny, int32_t row_lo, int32_t row_hi, int32_t lo_min, int32_t hi_max,
                               int32_t edge_top, int32_t edge_bot, int32_t sub_begin, int32_t sub_count,
                               int32_t n_sub, double coeff_dt, const double *uniform, int32_t part,
                               int32_t interior_passes, vk_stream_t stream) {
    if (part != VK_PART_ALL && part != VK_PART_INTERIOR && part != VK_PART_EDGES) {
        vk::set_error("vk_diffuse_part: part must be VK_PART_ALL / _INTERIOR / _EDGES");
        return VK_ERR_ARG;
    }
    if (part != VK_PART_ALL && !part_plan_ok(row_lo, row_hi, lo_min, hi_max, sub_count, edge_top, edge_bot)) {
        vk::set_error("vk_diffuse_part: the block is not a 10-deep-plan band block with an interior");
        return VK_ERR_LIMIT;
    }
    return diffuse_impl(field, work0, work1, n_fields, field_stride, ny, row_lo, row_hi, lo_min, hi_max, edge_top,
                        edge_bot, sub_begin, sub_count, n_sub, coeff_dt, uniform, part, interior_passes, stream);
}

static int diffuse_impl(double *field, double *work0, double *work1, int32_t n_fields, int64_t field_stride,
                        int32_t ny, int32_t row_lo, int32_t row_hi, int32_t lo_min, int32_t hi_max, int32_t edge_top,
                        int32_t edge_bot, int32_t sub_begin, int32_t sub_count, int32_t n_sub, double coeff_dt,
                        const double *uniform, int32_t part, int32_t split_m, vk_stream_t stream) {
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
    if (g_stencil_depth == 10 && sub_count % 10 == 0 && work1) {
        // A block of 10 k substeps: k passes of 10.  In the tolerance mode the final
        // pass writes the field without reading it back (no f0), so when the block ends
        // the step the field is a third buffer (its step-start values are not needed
        // once the first pass has read them).  The exact mode's final pass re-reads the
        // step-start field (f0 + (f - f0), in place like the odd-depth plan's), so there
        // the field is never scratch.  The block starts in the buffer the odd-depth
        // convention holds the state in (field for substep 0, else work[(j-1)&1]) and
        // ends in the one it expects after the block (field after the last substep,
        // else work[last & 1]), so halo exchanges between blocks (row bands) see the
        // usual buffers.  Buffers are assigned backwards from the target: each pass
        // writes one its source is not (a block inside the step starts and ends in the
        // same work buffer, so it needs an even number of passes; otherwise it takes
        // the odd-depth plan below).  Uniform planes skip every pass (nothing reads
        // the buffers they leave unwritten) and keep their field.
        const int P = sub_count / 10;
        const bool ends_step = last_in_call == n_sub - 1;
        double *S = sub_begin == 0 ? field : work[(sub_begin - 1) & 1];
        double *T = ends_step ? field : work[last_in_call & 1];
        double *cand[3] = {work0, work1, field};
        // the field is scratch only in a tolerance-mode block that ends the step
        const int nc = (ends_step && g_stencil_mode == 1) ? 3 : 2;
        double *dsts[64];
        bool ok = P >= 1 && P <= 64;
        for (int p = P - 1; ok && p >= 0; --p) {
            if (p == P - 1) {
                dsts[p] = T;
            } else {
                dsts[p] = nullptr;
                for (int c = 0; c < nc && !dsts[p]; ++c)
                    if (cand[c] != dsts[p + 1] && (p > 0 || cand[c] != S)) dsts[p] = cand[c];
                ok = dsts[p] != nullptr;
            }
        }
        ok = ok && dsts[0] != S;
        if (ok) {
            // part (vk_diffuse_part): the interior of pass p is the rows whose inputs at
            // the block's start are all owned -- [row_lo + 10 (p+1), row_hi - 10 (p+1)) on
            // a side with halo rows -- and the edges are the rest of the pass's rows.
            // The interior passes read and write only interior rows of each buffer, the
            // edge passes read at most 20 rows into the interior of the pass before, which
            // no later interior pass writes (it starts 10 rows deeper per pass), so the
            // interior of the first m passes can run before any edge pass (while the halo
            // arrives).  Then (part EDGES) the edges of those m passes, and the remaining
            // passes whole.
            const bool halo_top = !edge_top && row_lo > lo_min, halo_bot = !edge_bot && row_hi < hi_max;
            const int m = (split_m <= 0 || split_m > P) ? P : split_m;
            for (int p = 0; p < P; ++p) {
                if (part == VK_PART_INTERIOR && p >= m) break;
                const int e = sub_begin + 10 * p + 9;
                const int grow = last_in_call - e;
                const int lo = max(lo_min, row_lo - grow);
                const int hi = min(hi_max, row_hi + grow);
                const double *f0 = (g_stencil_mode != 1 && ends_step && p == P - 1) ? field : nullptr;
                const int ilo = halo_top ? row_lo + 10 * (p + 1) : lo;
                const int ihi = halo_bot ? row_hi - 10 * (p + 1) : hi;
                int ranges[3][2];
                int nr = 0;
                const bool strip = part == VK_PART_EDGES && p < m;
                if (part == VK_PART_ALL || (part == VK_PART_EDGES && p >= m)) {
                    ranges[nr][0] = lo, ranges[nr][1] = hi, ++nr;
                } else if (part == VK_PART_INTERIOR) {
                    ranges[nr][0] = ilo, ranges[nr][1] = ihi, ++nr;
                } else if (halo_top && halo_bot && ilo < ihi && g_stencil_mode == 1) {
                    // both strips as one launch (pair-sum pass with a row gap)
                    const int in_lo = max(lo_min, lo - 10), in_hi = min(hi_max, hi + 10);
                    vk_launch_ps10_strips(10, s, p ? dsts[p - 1] : S, dsts[p], f0, n_fields, field_stride, ny, lo, hi,
                                          in_lo, in_hi, top_reflect, bot_reflect, coeff_dt, uniform, nullptr, ilo, ihi);
                    int rc = vk::launch_check("vk_diffuse kernel (depth 10, edge strips)");
                    if (rc) return rc;
                } else {
                    if (halo_top) ranges[nr][0] = lo, ranges[nr][1] = ilo, ++nr;
                    if (halo_bot) ranges[nr][0] = ihi, ranges[nr][1] = hi, ++nr;
                }
                for (int q = 0; q < nr; ++q) {
                    const int olo = ranges[q][0], ohi = ranges[q][1];
                    if (olo >= ohi) continue;
                    const int in_lo = max(lo_min, olo - 10), in_hi = min(hi_max, ohi + 10);
                    launch_pass(10, s, p ? dsts[p - 1] : S, dsts[p], f0, n_fields, field_stride, ny, olo, ohi, in_lo,
                                in_hi, top_reflect, bot_reflect, coeff_dt, uniform, nullptr, strip);
                    int rc = vk::launch_check("vk_diffuse kernel (depth 10)");
                    if (rc) return rc;
                }
            }
            return VK_OK;
        }
        if (part != VK_PART_ALL) {
            vk::set_error("vk_diffuse_part: no 10-deep buffer plan for this block");
            return VK_ERR_LIMIT;
        }
    }
    if (part != VK_PART_ALL) {
        vk::set_error("vk_diffuse_part: only the 10-deep plan splits");
        return VK_ERR_LIMIT;
    }
    const std::vector<int> ks = odd_plan(sub_count);
    int j = sub_begin;
    for (size_t p = 0; p < ks.size(); ++p) {
        const int k = ks[p];
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
                               hi, top_reflect, bot_reflect, coeff_dt, uniform, 0);
        } else {
            launch_pass(k, s, src, dst, f0, n_fields, field_stride, ny, lo, hi, in_lo, in_hi, top_reflect, bot_reflect,
                        coeff_dt, uniform, nullptr);
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

// A whole-plane step's passes with the agent coupling inside them: the first
// pass also gathers each agent's external concentrations from the pre-step
// planes, the final pass also scatters the exchange into the new planes (one
// launch each less, and the exchange's read-modify-write of the planes happens
// while the final pass holds them).  Either arithmetic mode.  Returns
// VK_ERR_LIMIT, launching nothing, when the step is not planned as two or more
// fused passes.
extern "C" int vk_diffuse_coupled(double *field, double *work0, double *work1, int32_t n_fields,
                                  int64_t field_stride, int32_t ny, int32_t rows, int32_t n_sub, double coeff_dt,
                                  const double *uniform, const int32_t *bin_lin, const int32_t *seg, int32_t nseg,
                                  int64_t n_agents, const int32_t *gather_row, double *conc, int64_t conc_ld,
                                  const int32_t *count_row, const int64_t *counts, int64_t counts_ld,
                                  double binvol_avogadro, vk_stream_t stream) {
    if (!field || !work0 || !work1 || n_fields < 1 || ny <= 0 || rows <= 0 || n_sub < 0 ||
        (int64_t)rows * ny > field_stride || (int64_t)rows * ny >= INT32_MAX || n_agents < 0 ||
        n_agents >= INT32_MAX || nseg != (ny + 15) / 16 || (n_agents > 0 && (!bin_lin || !seg)) || !gather_row ||
        !count_row) {
        vk::set_error("vk_diffuse_coupled: bad arguments");
        return VK_ERR_ARG;
    }
    VkPsCouple cp = {};
    cp.bins = bin_lin;
    cp.seg = seg;
    cp.nseg = nseg;
    cp.n = (int32_t)n_agents;
    cp.gdst = conc;
    cp.gld = conc_ld;
    cp.counts = counts;
    cp.cld = counts_ld;
    cp.bva = binvol_avogadro;
    if (n_fields <= VK_COUPLE_MAX_FIELDS) {
        for (int f = 0; f < n_fields; ++f) {
            if (gather_row[f] >= 127 || count_row[f] >= 127 || (gather_row[f] >= 0 && (!conc || conc_ld < n_agents)) ||
                (count_row[f] >= 0 && (!counts || counts_ld < n_agents))) {
                vk::set_error("vk_diffuse_coupled: bad gather / count rows");
                return VK_ERR_ARG;
            }
            cp.grow[f] = (int8_t)(gather_row[f] < 0 ? -1 : gather_row[f]);
            cp.crow[f] = (int8_t)(count_row[f] < 0 ? -1 : count_row[f]);
        }
    }
    // the plan: vk_diffuse's (10-deep passes in the tolerance mode's depth-10 setting,
    // else odd depths), at least two fused passes (the gather rides on the first, the
    // exchange on the last) and no single-substep pass
    if (n_fields > VK_COUPLE_MAX_FIELDS || n_sub < 2) {
        vk::set_error("vk_diffuse_coupled: at most 8 planes and 2 substeps");
        return VK_ERR_LIMIT;
    }
    const bool ten = g_stencil_depth == 10 && g_stencil_mode == 1 && n_sub % 10 == 0 && n_sub >= 20;
    std::vector<int> ks = ten ? std::vector<int>(n_sub / 10, 10) : odd_plan(n_sub);
    bool ok = ks.size() >= 2;
    for (int k : ks) ok = ok && k >= 2;
    if (!ok) {
        vk::set_error("vk_diffuse_coupled: the step is not planned as two or more fused passes");
        return VK_ERR_LIMIT;
    }
    hipStream_t s = (hipStream_t)stream;
    const int np = (int)ks.size();
    const double *cur = field;
    for (int p = 0, j = 0; p < np; j += ks[p], ++p) {
        const bool last = p == np - 1;
        double *dst;
        if (last) dst = field;
        else if (ten) dst = cur == work0 ? work1 : work0;
        else dst = (j + ks[p] - 1) & 1 ? work1 : work0;   // work[e & 1], e = this pass's last substep
        VkPsCouple c = cp;
        c.mode = n_agents > 0 ? (p == 0 ? 1 : 0) | (last ? 2 : 0) : 0;
        // the exact mode's final pass re-reads the step-start plane: vk_diffuse's f0
        launch_pass(ks[p], s, cur, dst, last ? field : nullptr, n_fields, field_stride, ny, 0, rows, 0, rows, 0,
                    rows - 1, coeff_dt, uniform, &c);
        const int rc = vk::launch_check("vk_diffuse_coupled kernel");
        if (rc) return rc;
        cur = dst;
    }
    return VK_OK;
}

extern "C" int vk_diffuse_delta(double *field, double *work0, double *work1, double *delta, int32_t n_fields,
                                int64_t field_stride, int32_t ny, int32_t row_lo, int32_t row_hi, int32_t lo_min,
                                int32_t hi_max, int32_t edge_top, int32_t edge_bot, int32_t sub_begin,
                                int32_t sub_count, int32_t n_sub, double coeff_dt, const double *uniform,
                                vk_stream_t stream) {
    if (!delta || sub_count < 1 || sub_begin + sub_count != n_sub) {
        vk::set_error("vk_diffuse_delta: needs a delta buffer and the call must end at the last substep");
        return VK_ERR_ARG;
    }
    // substeps before the last: the ordinary passes, none of them final (n_sub + 1),
    // over one more row on each side (the last substep's neighbours) where there is one
    if (sub_count > 1) {
        const int rc = vk_diffuse(field, work0, work1, n_fields, field_stride, ny, std::max(lo_min, row_lo - 1),
                                  std::min(hi_max, row_hi + 1), lo_min, hi_max, edge_top, edge_bot, sub_begin,
                                  sub_count - 1, n_sub + 1, coeff_dt, uniform, stream);
        if (rc) return rc;
    }
    const int jl = n_sub - 1;
    double *work[2] = {work0, work1};
    const double *src = jl == 0 ? field : work[(jl - 1) & 1];
    const int top_reflect = edge_top ? lo_min : -1;
    const int bot_reflect = edge_bot ? hi_max - 1 : 0x7fffffff;
    dim3 grid((ny + ST_BX - 1) / ST_BX, (row_hi - row_lo + ST_RB - 1) / ST_RB, n_fields);
    hipLaunchKernelGGL(k_diffuse_substep, grid, dim3(ST_BX), 0, (hipStream_t)stream, src, delta, field, field_stride,
                       ny, row_lo, row_hi, top_reflect, bot_reflect, coeff_dt, uniform, 1);
    return vk::launch_check("vk_diffuse_delta");
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
                                                double *dst, int64_t ld) {
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
