// Internal helpers shared by the vk_* translation units (gfx950 / CDNA4 only).
#pragma once

#include <hip/hip_runtime.h>
#include <stdint.h>

#include "vk_kinetics.h"

// Device view of a compiled rate-law table.  Passed by value as a kernel
// argument (lands in the kernarg segment -> SGPRs).  Table walks are
// wave-uniform, so every table read goes through the scalar unit (ldc()).
struct vk_dev_table {
    const int32_t *ib;  // int32 arrays, concatenated
    const double *db;   // double arrays, concatenated
    int32_t n_species, n_dyn, n_reactions, n_rate_laws, n_params, n_ext;
    // element offsets of each array inside ib / db (one SGPR each)
    int32_t o_rl_reaction, o_rl_enzyme, o_rl_kcat, o_rl_num_ptr, o_rl_den_ptr;
    int32_t o_set_ptr, o_mem_species, o_mem_param, o_upd_ptr, o_upd_rxn, o_ex_ptr, o_ex_rxn;
    int32_t o_upd_coeff, o_ex_coeff;
    // reaction -> rate laws CSR (rate laws of reaction r in evaluation order),
    // derived from rl_reaction at vk_table_create; the wavefront kernel sums
    // flux[r] = 0 + v_l0 + v_l1 ... in the same order as the lane kernels
    int32_t o_rx_ptr, o_rx_rl;
};

struct vk_table {
    vk_dev_table dev;
    void *blob;  // single device allocation holding every array
    int32_t n_sets, n_members, n_upd, n_exch;
    int32_t n_ib, n_db;                    // element counts of the int / double blob parts
    hipModule_t spec_module = nullptr;     // vk_table_specialize (hiprtc)
    hipFunction_t spec_dopri5 = nullptr;      // agent per lane (variant 2)
    hipFunction_t spec_wave = nullptr;        // agent per wavefront (variant 3)
    int spec_wave_waves = 4;                  // its waves (agents) per workgroup: the launch bound / 64
    hipFunction_t spec_multi = nullptr;       // agent per lane, several steps per launch (vk_step_dopri5_multi)
    hipFunction_t spec_gather = nullptr;      // agent per lane + the next step's gather (vk_step_dopri5_gather)
};

// Load through the constant address space: uniform index -> s_load (scalar cache).
template <class T>
__device__ __forceinline__ T ldc(const T *p, int i) {
    return ((const __attribute__((address_space(4))) T *)p)[i];
}

// table element access: TI(t, set_ptr, i) == set_ptr[i] through the scalar cache
#define TI(t, arr, i) ldc((t).ib, (t).o_##arr + (i))
#define TD(t, arr, i) ldc((t).db, (t).o_##arr + (i))

namespace vk {
void set_error(const char *fmt, ...);
int hip_check(hipError_t e, const char *what);
int launch_check(const char *what);
}  // namespace vk
