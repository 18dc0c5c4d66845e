// Cell growth, derivers and division on MI355X (gfx950).
//
// Reference semantics (all per agent, per 1-s step):
//   GrowthProtein.next_update   vivarium/processes/growth_protein.py:88-107
//   Growth.next_update          vivarium/processes/growth.py:101-107
//   DivisionVolume.next_update  vivarium/processes/division_volume.py:39-45
//   TreeMass (calculate_mass)   vivarium/processes/tree_mass.py:10-18
//   DeriveGlobals.next_update   vivarium/processes/derive_globals.py:131-152 (+ :20-50)
//   MetaDivision / _divide      vivarium/processes/meta_division.py:15-88,
//                               vivarium/core/experiment.py:664-697
//   dividers                    vivarium/core/registry.py:197-280
// Compiled with -ffp-contract=off and written in the reference's operation
// order, so every float result is bit-identical to the reference's Python
// (the host evaluates exp(), pow() and the units' conversion factors with the
// same libraries the reference used and passes them in vk_cell_params).
//
// Division is a stable compaction: survivors keep their relative order and
// the two daughters of each mother are appended in mother order -- the agent
// order the reference's Store ends up with (daughters generated at the end of
// the agents dict, mother deleted).  The plan is one exclusive scan of the
// divide flags (block counts -> one-block scan -> per-block ranks); every SoA
// array is then gathered once into the new layout with its divider.

#include <stdint.h>

#include "vk_internal.h"

// ---------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al., SC'11), counter-based: u depends only on
// (seed, step, lineage), never on agent order or launch geometry.
// ---------------------------------------------------------------------------

__device__ __forceinline__ void philox_round(uint32_t (&c)[4], const uint32_t (&k)[2]) {
    const uint64_t p0 = (uint64_t)0xD2511F53u * c[0];
    const uint64_t p1 = (uint64_t)0xCD9E8D57u * c[2];
    const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
    const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
    c[0] = hi1 ^ c[1] ^ k[0];
    c[1] = lo1;
    c[2] = hi0 ^ c[3] ^ k[1];
    c[3] = lo0;
}

// uniform double in [0, 1) with 53 random bits, numpy's (a >> 5, b >> 6) construction
__device__ __forceinline__ double philox_uniform(uint64_t seed, uint64_t step, int32_t root, int32_t depth,
                                                 uint64_t path) {
    uint32_t c[4] = {(uint32_t)step, (uint32_t)root, (uint32_t)path, (uint32_t)(path >> 32)};
    uint32_t k[2] = {(uint32_t)seed + (uint32_t)depth, (uint32_t)(seed >> 32)};
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        if (r) {
            k[0] += 0x9E3779B9u;
            k[1] += 0xBB67AE85u;
        }
        philox_round(c, k);
    }
    const double a = (double)(c[0] >> 5), b = (double)(c[1] >> 6);
    return (a * 67108864.0 + b) / 9007199254740992.0;
}

// ---------------------------------------------------------------------------
// growth process + derivers
// ---------------------------------------------------------------------------

__global__ __launch_bounds__(256) void k_cell_step(vk_cell_params p, int64_t n, int64_t ld, double *__restrict__ cell,
                                                   double *__restrict__ m2c, const double *__restrict__ u,
                                                   const int32_t *__restrict__ root, const int32_t *__restrict__ depth,
                                                   const uint64_t *__restrict__ path, int32_t *__restrict__ divide) {
    const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= n) return;
    double *mass = cell + (int64_t)VK_CELL_MASS * ld + a;
    double *volume = cell + (int64_t)VK_CELL_VOLUME * ld + a;
    double *length = cell + (int64_t)VK_CELL_LENGTH * ld + a;
    double *area = cell + (int64_t)VK_CELL_SURFACE_AREA * ld + a;
    double *protein = cell + (int64_t)VK_CELL_PROTEIN * ld + a;
    int32_t div;
    double m;
    if (p.model == VK_GROWTH_PROTEIN) {
        // process, from the step-start protein
        const double pr = *protein;
        const double total = pr * p.factor;
        double added = trunc(total - pr);            // int(total - protein)
        const double extra = total - trunc(total);   // total - int(total)
        const double draw = (p.rng == VK_RNG_PHILOX)
                                ? philox_uniform(p.seed, p.step, root[a], depth[a], path[a])
                                : u[a];
        if (draw < extra) added = added + 1.0;
        div = pr >= p.divide_protein;
        const double pn = pr + added;
        *protein = pn;
        // mass_deriver: 0 fg + mw * (count / N_A), g -> fg
        m = 0.0 + (p.protein_mw * (pn / p.avogadro)) * p.fg_per_g;
    } else {
        div = *volume >= p.division_volume;          // DivisionVolume, step-start volume
        m = *mass * p.factor;                         // Growth
    }
    *mass = m;
    // globals_deriver: volume = mass / density (magnitude), then .to('fL')
    const double raw = m / p.density;
    *volume = raw * p.volume_to_fl;
    m2c[a] = p.avogadro * (raw * 1e-15) * 1e-3;
    const double len = (raw - p.cap_volume) / p.cap_area + p.two_r;
    *length = len;
    *area = p.sa_const + p.sa_lin * (len - p.width);
    divide[a] = div;
}

extern "C" int vk_cell_step(const vk_cell_params *p, int64_t n, int64_t ld, double *cell, double *m2c,
                            const double *u, const int32_t *root, const int32_t *depth, const uint64_t *path,
                            int32_t *divide, vk_stream_t stream) {
    if (!p || n < 0 || ld < n || (n > 0 && (!cell || !m2c || !divide))) {
        vk::set_error("vk_cell_step: bad arguments");
        return VK_ERR_ARG;
    }
    if (p->model != VK_GROWTH_PROTEIN && p->model != VK_GROWTH_MASS) {
        vk::set_error("vk_cell_step: unknown growth model %d", p->model);
        return VK_ERR_ARG;
    }
    if (p->model == VK_GROWTH_PROTEIN && n > 0) {
        if (p->rng == VK_RNG_STREAM && !u) {
            vk::set_error("vk_cell_step: VK_RNG_STREAM needs u[]");
            return VK_ERR_ARG;
        }
        if (p->rng == VK_RNG_PHILOX && (!root || !depth || !path)) {
            vk::set_error("vk_cell_step: VK_RNG_PHILOX needs the lineage arrays");
            return VK_ERR_ARG;
        }
        if (p->rng != VK_RNG_STREAM && p->rng != VK_RNG_PHILOX) {
            vk::set_error("vk_cell_step: unknown rng %d", p->rng);
            return VK_ERR_ARG;
        }
    }
    if (n == 0) return VK_OK;
    hipLaunchKernelGGL(k_cell_step, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *p, n,
                       ld, cell, m2c, u, root, depth, path, divide);
    return vk::launch_check("k_cell_step");
}

// ---------------------------------------------------------------------------
// division plan: exclusive scan of the divide flags
// ---------------------------------------------------------------------------

constexpr int DV_BLOCK = 1024;   // agents per scan block (256 threads x 4)

int64_t vk_divide_scratch_bytes_impl(int64_t n) {
    const int64_t nb = (n + DV_BLOCK - 1) / DV_BLOCK;
    return (nb + 2) * (int64_t)sizeof(int64_t);
}

extern "C" int64_t vk_divide_scratch_bytes(int64_t n) { return n < 0 ? 0 : vk_divide_scratch_bytes_impl(n); }

__global__ __launch_bounds__(256) void k_divide_count(const int32_t *__restrict__ divide, int64_t n,
                                                      int64_t *__restrict__ block_count) {
    const int64_t base = (int64_t)blockIdx.x * DV_BLOCK;
    int c = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t a = base + k * 256 + threadIdx.x;
        if (a < n && divide[a]) ++c;
    }
    __shared__ int part[4];
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = c;
    __syncthreads();
    if (threadIdx.x == 0) block_count[blockIdx.x] = part[0] + part[1] + part[2] + part[3];
}

// one block: exclusive scan of nb block counts in place; total -> *total, n + total -> *n_out
__global__ __launch_bounds__(256) void k_divide_scan_blocks(int64_t *__restrict__ block_count, int64_t nb,
                                                            int64_t n, int64_t *__restrict__ n_out) {
    __shared__ int64_t carry;
    __shared__ int64_t wsum[4];
    if (threadIdx.x == 0) carry = 0;
    __syncthreads();
    for (int64_t b0 = 0; b0 < nb; b0 += 256) {
        const int64_t b = b0 + threadIdx.x;
        const int64_t v = b < nb ? block_count[b] : 0;
        // inclusive wave scan
        int64_t x = v;
        const int lane = threadIdx.x & 63;
#pragma unroll
        for (int o = 1; o < 64; o <<= 1) {
            const int64_t y = __shfl_up(x, o);
            if (lane >= o) x += y;
        }
        if (lane == 63) wsum[threadIdx.x >> 6] = x;
        __syncthreads();
        int64_t wo = 0;
        for (int w = 0; w < (int)(threadIdx.x >> 6); ++w) wo += wsum[w];
        const int64_t excl = carry + wo + x - v;
        __syncthreads();
        if (b < nb) block_count[b] = excl;
        if (threadIdx.x == 255) carry = excl + v;
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        block_count[nb] = carry;   // total number of mothers
        *n_out = n + carry;
    }
}

__global__ __launch_bounds__(256) void k_divide_place(const int32_t *__restrict__ divide, int64_t n,
                                                      const int64_t *__restrict__ block_off, int64_t nb,
                                                      int32_t *__restrict__ src_index, int32_t *__restrict__ kind) {
    const int64_t base = (int64_t)blockIdx.x * DV_BLOCK;
    const int64_t total = block_off[nb];
    const int64_t n_keep = n - total;
    __shared__ int wcount[16];
    // per-thread 4 consecutive agents -> thread-level counts -> block exclusive scan
    const int64_t a0 = base + (int64_t)threadIdx.x * 4;
    int f[4], c = 0;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        f[k] = (a0 + k < n) ? (divide[a0 + k] != 0) : 0;
        c += f[k];
    }
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int x = c;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1) {
        const int y = __shfl_up(x, o);
        if (lane >= o) x += y;
    }
    if (lane == 63) wcount[w] = x;
    __syncthreads();
    int wo = 0;
    for (int k = 0; k < w; ++k) wo += wcount[k];
    int64_t m = block_off[blockIdx.x] + wo + x - c;   // mothers before a0
#pragma unroll
    for (int k = 0; k < 4; ++k) {
        const int64_t a = a0 + k;
        if (a >= n) break;
        if (f[k]) {
            const int64_t j = n_keep + 2 * m;
            src_index[j] = (int32_t)a;
            kind[j] = 0;
            src_index[j + 1] = (int32_t)a;
            kind[j + 1] = 1;
            ++m;
        } else {
            const int64_t j = a - m;
            src_index[j] = (int32_t)a;
            kind[j] = -1;
        }
    }
}

extern "C" int vk_divide_plan(const int32_t *divide, int64_t n, int32_t *src_index, int32_t *kind, int64_t *n_out,
                              void *scratch, vk_stream_t stream) {
    if (n < 0 || n > 0x3fffffff || !n_out || !scratch || (n > 0 && (!divide || !src_index || !kind))) {
        vk::set_error("vk_divide_plan: bad arguments");
        return VK_ERR_ARG;
    }
    hipStream_t s = (hipStream_t)stream;
    int64_t *bc = (int64_t *)scratch;
    const int64_t nb = (n + DV_BLOCK - 1) / DV_BLOCK;
    if (nb > 0)
        hipLaunchKernelGGL(k_divide_count, dim3((unsigned)nb), dim3(256), 0, s, divide, n, bc);
    hipLaunchKernelGGL(k_divide_scan_blocks, dim3(1), dim3(256), 0, s, bc, nb, n, n_out);
    if (nb > 0)
        hipLaunchKernelGGL(k_divide_place, dim3((unsigned)nb), dim3(256), 0, s, divide, n, bc, nb, src_index, kind);
    return vk::launch_check("vk_divide_plan");
}

// ---------------------------------------------------------------------------
// gathers with dividers
// ---------------------------------------------------------------------------

template <typename T, int DIV>
__global__ __launch_bounds__(256) void k_divide_gather(int64_t n_out, const int32_t *__restrict__ src_index,
                                                       const int32_t *__restrict__ kind, const T *__restrict__ src,
                                                       int64_t ld_src, T *__restrict__ dst, int64_t ld_dst, int rows) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_out) return;
    const int64_t a = src_index[j];
    const bool daughter = kind[j] >= 0;
    for (int r = 0; r < rows; ++r) {
        T v = src[(int64_t)r * ld_src + a];
        if (daughter) {
            if constexpr (DIV == VK_DIVIDE_SPLIT) v = v / (T)2;
            if constexpr (DIV == VK_DIVIDE_ZERO) v = (T)0;
        }
        dst[(int64_t)r * ld_dst + j] = v;
    }
}

extern "C" int vk_divide_gather(int64_t n_out, const int32_t *src_index, const int32_t *kind, const void *src,
                                int64_t ld_src, void *dst, int64_t ld_dst, int32_t rows, int32_t elem_bytes,
                                int32_t divider, vk_stream_t stream) {
    if (n_out < 0 || ld_dst < n_out || rows < 0 || (n_out > 0 && rows > 0 && (!src || !dst || !src_index || !kind)) ||
        (elem_bytes != 4 && elem_bytes != 8) || divider < 0 || divider > 2 ||
        (divider == VK_DIVIDE_SPLIT && elem_bytes != 8)) {
        vk::set_error("vk_divide_gather: bad arguments");
        return VK_ERR_ARG;
    }
    if (n_out == 0 || rows == 0) return VK_OK;
    hipStream_t s = (hipStream_t)stream;
    const dim3 g((unsigned)((n_out + 255) / 256)), b(256);
#define VK_G(T, D) hipLaunchKernelGGL((k_divide_gather<T, D>), g, b, 0, s, n_out, src_index, kind, (const T *)src, ld_src, (T *)dst, ld_dst, rows)
    if (elem_bytes == 8) {
        if (divider == VK_DIVIDE_SET) VK_G(double, VK_DIVIDE_SET);
        else if (divider == VK_DIVIDE_SPLIT) VK_G(double, VK_DIVIDE_SPLIT);
        else VK_G(double, VK_DIVIDE_ZERO);
    } else {
        if (divider == VK_DIVIDE_SET) VK_G(int32_t, VK_DIVIDE_SET);
        else VK_G(int32_t, VK_DIVIDE_ZERO);
    }
#undef VK_G
    return vk::launch_check("k_divide_gather");
}

__global__ __launch_bounds__(256) void k_divide_lineage(int64_t n_out, const int32_t *__restrict__ src_index,
                                                        const int32_t *__restrict__ kind,
                                                        const int32_t *__restrict__ root_src,
                                                        const int32_t *__restrict__ depth_src,
                                                        const uint64_t *__restrict__ path_src,
                                                        int32_t *__restrict__ root_dst, int32_t *__restrict__ depth_dst,
                                                        uint64_t *__restrict__ path_dst, int32_t *overflow) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_out) return;
    const int64_t a = src_index[j];
    const int k = kind[j];
    int32_t d = depth_src[a];
    uint64_t pth = path_src[a];
    if (k >= 0) {
        if (d >= 64 && overflow) *overflow = 1;
        pth = (pth << 1) | (uint64_t)k;
        d = d + 1;
    }
    root_dst[j] = root_src[a];
    depth_dst[j] = d;
    path_dst[j] = pth;
}

extern "C" int vk_divide_lineage(int64_t n_out, const int32_t *src_index, const int32_t *kind, const int32_t *root_src,
                                 const int32_t *depth_src, const uint64_t *path_src, int32_t *root_dst,
                                 int32_t *depth_dst, uint64_t *path_dst, int32_t *overflow, vk_stream_t stream) {
    if (n_out < 0 || (n_out > 0 && (!src_index || !kind || !root_src || !depth_src || !path_src || !root_dst ||
                                    !depth_dst || !path_dst))) {
        vk::set_error("vk_divide_lineage: bad arguments");
        return VK_ERR_ARG;
    }
    if (n_out == 0) return VK_OK;
    hipLaunchKernelGGL(k_divide_lineage, dim3((unsigned)((n_out + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       n_out, src_index, kind, root_src, depth_src, path_src, root_dst, depth_dst, path_dst, overflow);
    return vk::launch_check("k_divide_lineage");
}

__global__ __launch_bounds__(256) void k_divide_locations(int64_t n_out, const int32_t *__restrict__ src_index,
                                                          const int32_t *__restrict__ kind,
                                                          const double *__restrict__ loc_src, int64_t ld_src,
                                                          double *__restrict__ loc_dst, int64_t ld_dst,
                                                          const double *__restrict__ cell_dst) {
    const int64_t j = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (j >= n_out) return;
    const int64_t a = src_index[j];
    const int k = kind[j];
    double x = loc_src[a], y = loc_src[ld_src + a];
    if (k >= 0) {
        // parent values: length was split into this slot (exact halving), angle copied
        const double parent_length = cell_dst[(int64_t)VK_CELL_LENGTH * ld_dst + j] * 2.0;
        const double angle = cell_dst[(int64_t)VK_CELL_ANGLE * ld_dst + j];
        const double ratio = k == 0 ? -0.25 : 0.25;
        const double dx = parent_length * ratio * cos(angle);
        const double dy = parent_length * ratio * sin(angle);
        x = x + dx;
        y = y + dy;
    }
    loc_dst[j] = x;
    loc_dst[ld_dst + j] = y;
}

extern "C" int vk_divide_locations(int64_t n_out, const int32_t *src_index, const int32_t *kind, const double *loc_src,
                                   int64_t ld_src, double *loc_dst, int64_t ld_dst, const double *cell_dst,
                                   vk_stream_t stream) {
    if (n_out < 0 || ld_dst < n_out || (n_out > 0 && (!src_index || !kind || !loc_src || !loc_dst || !cell_dst))) {
        vk::set_error("vk_divide_locations: bad arguments");
        return VK_ERR_ARG;
    }
    if (n_out == 0) return VK_OK;
    hipLaunchKernelGGL(k_divide_locations, dim3((unsigned)((n_out + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       n_out, src_index, kind, loc_src, ld_src, loc_dst, ld_dst, cell_dst);
    return vk::launch_check("k_divide_locations");
}
