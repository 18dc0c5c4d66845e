// Launchers of the fused-pass stencil kernels (vk_stencil_*.hip), called by
// vk_diffuse (vk_lattice.hip).  k = substeps fused in the pass (odd, 3..15);
// f0 != nullptr marks the FINAL pass (writes f0 + (f - f0)).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#define VK_STENCIL_LAUNCH_ARGS                                                                                 \
    int k, hipStream_t st, const double *src, double *dst, const double *f0, int nf, int64_t fs, int ny,        \
        int out_lo, int out_hi, int in_lo, int in_hi, int top, int bot, double coef, const double *mm,          \
        const struct VkPsCouple *cp

extern int g_stencil_rows;   // output rows per wave tile, 0 = auto (vk_lattice.hip, vk_set_stencil_kernel)
extern int g_stencil_mode;   // 0 = bit-exact (default), 1 = tolerance / FMA (vk_set_stencil_mode)

struct VkPsCouple;
void vk_launch_wl3(VK_STENCIL_LAUNCH_ARGS);          // lag-1 wave tile, 3 rows prefetched
void vk_launch_wl6(VK_STENCIL_LAUNCH_ARGS);          // lag-1 wave tile, 6 rows prefetched
void vk_launch_wl6nt(VK_STENCIL_LAUNCH_ARGS);        // as wl6 with streaming stores (k = 7, 9, 11; 10 tolerance mode)
// Agent coupling carried by a pair-sum pass (vk_diffuse_coupled): each wave
// handles the agents whose bins lie in its own output rows x columns.  Agents
// are stored in bin order (bins ascending); seg[r * nseg + s] = the first agent
// with bin >= r * ny + 16 s.
#define VK_COUPLE_MAX_FIELDS 8
struct VkPsCouple {
    const int32_t *bins;
    const int32_t *seg;
    int32_t nseg;
    int32_t n;                             // agents
    int32_t mode;                          // bit 0: gather before the pass, bit 1: exchange after it
    double *gdst;                          // gather: gdst[grow[f] * gld + a] = plane f at bins[a] (pre-pass)
    int64_t gld;
    const int64_t *counts;                 // exchange: plane f += counts[crow[f] * cld + a] / bva * 1000
    int64_t cld;
    double bva;
    int8_t grow[VK_COUPLE_MAX_FIELDS];     // -1 = none
    int8_t crow[VK_COUPLE_MAX_FIELDS];
};

void vk_launch_ps(VK_STENCIL_LAUNCH_ARGS);     // tolerance mode, pair-sum form (k = 3, 5, 7, 9, 11)
void vk_launch_ps10(VK_STENCIL_LAUNCH_ARGS);   // the same, k = 10
void vk_launch_ps10_strips(VK_STENCIL_LAUNCH_ARGS, int gap_lo, int gap_hi);   // k = 10, two strips
void vk_launch_ps10_aligned(VK_STENCIL_LAUNCH_ARGS);   // k = 10, 96 written columns (variant 70)
bool vk_launch_sp(int variant, VK_STENCIL_LAUNCH_ARGS);       // variant 40-43 (k = 10); false: not taken

// ---------------------------------------------------------------------------
// Agent coupling inside a pass (vk_diffuse_coupled), shared by both kernel
// families.  A wave owns the cells of its output rows [c0, c1) x columns
// [x0, x0 + W); agents are stored in bin order, so the agents of one such row
// segment are a contiguous run found from the 16-column index cp.seg.  One lane
// per row; each lane takes its run in batches of VK_COUPLE_BATCH agents, issuing
// a batch's loads together (the run is ~7 agents at C4), so a wave waits about
// two load latencies, not one per agent.
// ---------------------------------------------------------------------------
#define VK_COUPLE_BATCH 16

// The first pass: gdst[grow[f] * gld + a] = the pre-step plane at bins[a]
// (get_local_environments, diffusion_field.py:362-379), read before any pass
// has written the plane -- the first pass reads `field` and writes a work buffer.
__device__ __forceinline__ void vk_couple_gather(const VkPsCouple &cp, const double *plane, int f, int ny, int x0,
                                                 int W, int c0, int c1, int lane) {
    const int g = cp.grow[f];
    if (g < 0) return;
    double *dst = cp.gdst + (int64_t)g * cp.gld;
    const int ce = min(x0 + W, ny);
    for (int r = c0 + lane; r < c1; r += 64) {
        const int bb = r * ny + x0, be = r * ny + ce;
        int a = cp.seg[(int64_t)r * cp.nseg + (x0 >> 4)];
        for (;;) {
            int b[VK_COUPLE_BATCH];
#pragma unroll
            for (int j = 0; j < VK_COUPLE_BATCH; ++j) b[j] = a + j < cp.n ? cp.bins[a + j] : 0x7fffffff;
            double v[VK_COUPLE_BATCH];
#pragma unroll
            for (int j = 0; j < VK_COUPLE_BATCH; ++j) v[j] = (b[j] >= bb && b[j] < be) ? plane[b[j]] : 0.0;
#pragma unroll
            for (int j = 0; j < VK_COUPLE_BATCH; ++j)
                if (b[j] >= bb && b[j] < be) dst[a + j] = v[j];
            if (b[VK_COUPLE_BATCH - 1] >= be) break;
            a += VK_COUPLE_BATCH;
        }
    }
}

// The final pass, after the wave's own stores: for each cell of the segment,
// plane += counts[crow[f] * cld + a] / bva * 1000 for its agents in agent order
// (update_field_with_exchange, registry.py:149-183, applied agent by agent as
// k_exchange_sorted does -- the same bits).  The stores were made by other lanes
// of this wave: a workgroup-scope fence orders them before the loads, which go
// to L2 (agent-scope atomic loads skip the vector L1).
__device__ __forceinline__ void vk_couple_exchange(const VkPsCouple &cp, double *plane, int f, int ny, int x0, int W,
                                                   int c0, int c1, int lane) {
    const int cr = cp.crow[f];
    if (cr < 0) return;
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "workgroup");
    const int64_t *cnt = cp.counts + (int64_t)cr * cp.cld;
    const int ce = min(x0 + W, ny);
    for (int r = c0 + lane; r < c1; r += 64) {
        const int bb = r * ny + x0, be = r * ny + ce;
        int a = cp.seg[(int64_t)r * cp.nseg + (x0 >> 4)];
        int cur = -1;            // the cell being accumulated (its run may cross batches)
        double acc = 0.0;
        for (;;) {
            int b[VK_COUPLE_BATCH];
            int64_t c[VK_COUPLE_BATCH];
#pragma unroll
            for (int j = 0; j < VK_COUPLE_BATCH; ++j) {
                const bool in = a + j < cp.n;
                b[j] = in ? cp.bins[a + j] : 0x7fffffff;
                c[j] = in ? cnt[a + j] : 0;
            }
            double v[VK_COUPLE_BATCH];   // the plane at each agent's cell (used by the first agent of a run)
#pragma unroll
            for (int j = 0; j < VK_COUPLE_BATCH; ++j)
                v[j] = (b[j] >= bb && b[j] < be && b[j] != (j ? b[j - 1] : cur))
                           ? __hip_atomic_load(plane + b[j], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                           : 0.0;
#pragma unroll
            for (int j = 0; j < VK_COUPLE_BATCH; ++j) {
                if (b[j] >= bb && b[j] < be) {
                    if (b[j] != cur) {
                        if (cur >= 0) plane[cur] = acc;
                        cur = b[j];
                        acc = v[j];
                    }
                    acc = acc + ((double)c[j] / cp.bva) * 1000.0;
                }
            }
            if (b[VK_COUPLE_BATCH - 1] >= be) break;
            a += VK_COUPLE_BATCH;
        }
        if (cur >= 0) plane[cur] = acc;
    }
}
