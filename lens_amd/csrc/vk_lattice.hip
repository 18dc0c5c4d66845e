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
                                                           const double *__restrict__ minmax) {
    const int f = blockIdx.z;
    if (minmax && minmax[2 * f] == minmax[2 * f + 1]) return;  // uniform: delta is zero
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

extern "C" int vk_diffuse(double *field, double *work0, double *work1, int32_t n_fields,
                          int64_t field_stride, int32_t ny, int32_t row_lo, int32_t row_hi, int32_t lo_min,
                          int32_t hi_max, int32_t edge_top, int32_t edge_bot, int32_t sub_begin,
                          int32_t sub_count, int32_t n_sub, double coeff_dt, const double *minmax,
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
    double *work[2] = {work0, work1};
    const int top_reflect = edge_top ? lo_min : -1;
    const int bot_reflect = edge_bot ? hi_max - 1 : 0x7fffffff;
    hipStream_t s = (hipStream_t)stream;
    const int last_in_call = sub_begin + sub_count - 1;
    for (int jsub = sub_begin; jsub <= last_in_call; ++jsub) {
        const int grow = last_in_call - jsub;
        const int lo = max(lo_min, row_lo - grow);
        const int hi = min(hi_max, row_hi + grow);
        const double *src = (jsub == 0) ? field : work[(jsub - 1) & 1];
        const bool final_sub = (jsub == n_sub - 1);
        // a single-substep step cannot update `field` in place (neighbours
        // would read new values): it goes through work0 and is copied back
        const bool in_place = final_sub && jsub == 0;
        double *dst = (final_sub && !in_place) ? field : work[jsub & 1];
        const double *f0 = final_sub ? field : nullptr;
        dim3 grid((ny + ST_BX - 1) / ST_BX, (hi - lo + ST_RB - 1) / ST_RB, n_fields);
        hipLaunchKernelGGL(k_diffuse_substep, grid, dim3(ST_BX), 0, s, src, dst, f0, field_stride, ny, lo, hi,
                           top_reflect, bot_reflect, coeff_dt, minmax);
        if (in_place) {
            int rc = vk::launch_check("k_diffuse_substep");
            if (rc) return rc;
            for (int f = 0; f < n_fields; ++f) {
                const int64_t off = (int64_t)f * field_stride + (int64_t)row_lo * ny;
                rc = vk::hip_check(hipMemcpyAsync(field + off, work0 + off,
                                                  (size_t)(row_hi - row_lo) * ny * sizeof(double),
                                                  hipMemcpyDeviceToDevice, s), "hipMemcpyAsync(diffuse)");
                if (rc) return rc;
            }
        }
    }
    return vk::launch_check("k_diffuse_substep");
}

// ---------------------------------------------------------------------------
// min / max per plane (uniform-field test; multi-rank callers all-reduce)
// ---------------------------------------------------------------------------

__global__ void k_minmax_init(double *mm, int n_fields) {
    const int i = threadIdx.x;
    if (i < n_fields) {
        mm[2 * i] = INFINITY;
        mm[2 * i + 1] = -INFINITY;
    }
}

__global__ __launch_bounds__(256) void k_minmax(const double *__restrict__ fields, int64_t field_stride,
                                                int64_t off, int64_t count, double *mm) {
    const int f = blockIdx.y;
    const double *p = fields + (int64_t)f * field_stride + off;
    double lo = INFINITY, hi = -INFINITY;
    for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < count;
         i += (int64_t)gridDim.x * blockDim.x) {
        const double v = p[i];
        lo = fmin(lo, v);
        hi = fmax(hi, v);
    }
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) {
        lo = fmin(lo, __shfl_xor(lo, o));
        hi = fmax(hi, __shfl_xor(hi, o));
    }
    __shared__ double slo[4], shi[4];
    const int w = threadIdx.x >> 6;
    if ((threadIdx.x & 63) == 0) {
        slo[w] = lo;
        shi[w] = hi;
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        for (int k = 1; k < (int)(blockDim.x >> 6); ++k) {
            lo = fmin(lo, slo[k]);
            hi = fmax(hi, shi[k]);
        }
        __hip_atomic_fetch_min(&mm[2 * f], lo, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_fetch_max(&mm[2 * f + 1], hi, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
}

extern "C" int vk_field_minmax(const double *fields, int32_t n_fields, int64_t field_stride, int32_t ny,
                               int32_t row_lo, int32_t row_hi, double *minmax, vk_stream_t stream) {
    if (!fields || !minmax || n_fields < 0 || n_fields > 1024 || ny <= 0 || row_lo < 0 || row_hi < row_lo ||
        (int64_t)row_hi * ny > field_stride) {
        vk::set_error("vk_field_minmax: bad arguments");
        return VK_ERR_ARG;
    }
    if (n_fields == 0) return VK_OK;
    hipStream_t s = (hipStream_t)stream;
    hipLaunchKernelGGL(k_minmax_init, dim3(1), dim3(1024), 0, s, minmax, n_fields);
    const int64_t count = (int64_t)(row_hi - row_lo) * ny;
    if (count > 0) {
        const unsigned blocks = (unsigned)std::min<int64_t>(1024, (count + 255) / 256);
        hipLaunchKernelGGL(k_minmax, dim3(blocks, n_fields), dim3(256), 0, s, fields, field_stride,
                           (int64_t)row_lo * ny, count, minmax);
    }
    return vk::launch_check("k_minmax");
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
