// Batched convenience kinetics on MI355X (gfx950): rate-law table, reference
// Euler step and adaptive Dormand-Prince 5(4), one agent per lane.
//
// Reference semantics: vivarium/library/kinetic_rate_laws.py:149-178 (rate
// law), :277-297 (get_fluxes); vivarium/processes/convenience_kinetics.py:
// 303-352 (Euler step + integer exchange counts).  Compiled with
// -ffp-contract=off: the exact kernels reproduce the reference's Python
// floating-point operation order bit for bit; the DP45 kernel uses explicit
// fma() where it wants one.
//
// Layout: agent state is SoA, row stride ld, so lane a of a wave touches
// consecutive addresses for every row (coalesced 8-B-per-lane accesses).
// The table is identical for every lane, so its walk is wave-uniform and is
// read through the scalar cache (ldc()) -- no VGPRs, no LDS traffic.
// The ODE kernel keeps each lane's species vector as a column of an LDS
// tile (row s at lds[s*BS + lane]) because the rate laws index species at
// run time; the integrator's stage vectors stay in VGPRs (static indices).

#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <string.h>

#include <hip/hiprtc.h>

#include <algorithm>
#include <vector>

#include "vk_internal.h"

namespace vk {

static thread_local char g_err[512] = "";

void set_error(const char *fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof(g_err), fmt, ap);
    va_end(ap);
}

int hip_check(hipError_t e, const char *what) {
    if (e == hipSuccess) return VK_OK;
    set_error("%s: %s", what, hipGetErrorString(e));
    return VK_ERR_HIP;
}

int launch_check(const char *what) { return hip_check(hipGetLastError(), what); }

}  // namespace vk

extern "C" int vk_abi_version(void) { return VK_ABI_VERSION; }
extern "C" const char *vk_last_error(void) { return vk::g_err; }

// ---------------------------------------------------------------------------
// table management
// ---------------------------------------------------------------------------

extern "C" int vk_table_create(const vk_table_desc *d, vk_table **out) {
    if (!d || !out) {
        vk::set_error("vk_table_create: null argument");
        return VK_ERR_ARG;
    }
    *out = nullptr;
    if (d->n_species < 0 || d->n_dyn < 0 || d->n_dyn > d->n_species || d->n_reactions < 0 ||
        d->n_rate_laws < 0 || d->n_params < 0 || d->n_ext < 0 || d->n_sets < 0 ||
        d->n_members < 0 || d->n_upd < 0 || d->n_exch < 0) {
        vk::set_error("vk_table_create: negative or inconsistent sizes");
        return VK_ERR_ARG;
    }
    // validate every index on the host: a bad table must never reach a kernel
    auto bad = [&](const char *what) {
        vk::set_error("vk_table_create: invalid %s", what);
        return VK_ERR_ARG;
    };
    const int L = d->n_rate_laws;
    for (int l = 0; l < L; ++l) {
        if (d->rl_reaction[l] < 0 || d->rl_reaction[l] >= d->n_reactions) return bad("rl_reaction");
        if (d->rl_enzyme[l] < 0 || d->rl_enzyme[l] >= d->n_species) return bad("rl_enzyme");
        if (d->rl_kcat[l] < 0 || d->rl_kcat[l] >= d->n_params) return bad("rl_kcat");
    }
    for (int l = 0; l <= L; ++l) {
        if (d->rl_num_ptr[l] < 0 || d->rl_num_ptr[l] > d->n_sets) return bad("rl_num_ptr");
        if (d->rl_den_ptr[l] < 0 || d->rl_den_ptr[l] > d->n_sets) return bad("rl_den_ptr");
        if (l && (d->rl_num_ptr[l] < d->rl_num_ptr[l - 1] || d->rl_den_ptr[l] < d->rl_den_ptr[l - 1]))
            return bad("set pointers (not monotone)");
    }
    for (int s = 0; s <= d->n_sets; ++s) {
        if (d->set_ptr[s] < 0 || d->set_ptr[s] > d->n_members) return bad("set_ptr");
        if (s && d->set_ptr[s] < d->set_ptr[s - 1]) return bad("set_ptr (not monotone)");
    }
    for (int m = 0; m < d->n_members; ++m) {
        if (d->mem_species[m] < 0 || d->mem_species[m] >= d->n_species) return bad("mem_species");
        if (d->mem_param[m] < 0 || d->mem_param[m] >= d->n_params) return bad("mem_param");
    }
    for (int i = 0; i <= d->n_dyn; ++i)
        if (d->upd_ptr[i] < 0 || d->upd_ptr[i] > d->n_upd || (i && d->upd_ptr[i] < d->upd_ptr[i - 1]))
            return bad("upd_ptr");
    for (int j = 0; j < d->n_upd; ++j)
        if (d->upd_rxn[j] < 0 || d->upd_rxn[j] >= d->n_reactions) return bad("upd_rxn");
    for (int i = 0; i <= d->n_ext; ++i)
        if (d->ex_ptr[i] < 0 || d->ex_ptr[i] > d->n_exch || (i && d->ex_ptr[i] < d->ex_ptr[i - 1]))
            return bad("ex_ptr");
    for (int j = 0; j < d->n_exch; ++j)
        if (d->ex_rxn[j] < 0 || d->ex_rxn[j] >= d->n_reactions) return bad("ex_rxn");

    // one blob: doubles first (8-B aligned), then int32 arrays
    std::vector<double> dbl;
    dbl.insert(dbl.end(), d->upd_coeff, d->upd_coeff + d->n_upd);
    dbl.insert(dbl.end(), d->ex_coeff, d->ex_coeff + d->n_exch);
    std::vector<int32_t> ints;
    // reaction -> rate-law CSR (stable: evaluation order within a reaction)
    std::vector<int32_t> rx_ptr(d->n_reactions + 1, 0), rx_rl(L);
    for (int l = 0; l < L; ++l) rx_ptr[d->rl_reaction[l] + 1]++;
    for (int r = 0; r < d->n_reactions; ++r) rx_ptr[r + 1] += rx_ptr[r];
    {
        std::vector<int32_t> fill(rx_ptr.begin(), rx_ptr.end() - 1);
        for (int l = 0; l < L; ++l) rx_rl[fill[d->rl_reaction[l]]++] = l;
    }
    struct Seg { const int32_t *src; size_t n; size_t off; };
    Seg segs[] = {
        {d->rl_reaction, (size_t)L, 0}, {d->rl_enzyme, (size_t)L, 0}, {d->rl_kcat, (size_t)L, 0},
        {d->rl_num_ptr, (size_t)L + 1, 0}, {d->rl_den_ptr, (size_t)L + 1, 0},
        {d->set_ptr, (size_t)d->n_sets + 1, 0}, {d->mem_species, (size_t)d->n_members, 0},
        {d->mem_param, (size_t)d->n_members, 0}, {d->upd_ptr, (size_t)d->n_dyn + 1, 0},
        {d->upd_rxn, (size_t)d->n_upd, 0}, {d->ex_ptr, (size_t)d->n_ext + 1, 0},
        {d->ex_rxn, (size_t)d->n_exch, 0},
        {rx_ptr.data(), rx_ptr.size(), 0}, {rx_rl.data(), rx_rl.size(), 0},
    };
    for (auto &s : segs) {
        s.off = ints.size();
        ints.insert(ints.end(), s.src, s.src + s.n);
    }
    size_t dbytes = dbl.size() * sizeof(double);
    size_t bytes = dbytes + ints.size() * sizeof(int32_t) + 16;
    void *blob = nullptr;
    int rc = vk::hip_check(hipMalloc(&blob, bytes), "hipMalloc(table)");
    if (rc) return rc;
    if (!dbl.empty()) {
        rc = vk::hip_check(hipMemcpy(blob, dbl.data(), dbytes, hipMemcpyHostToDevice), "hipMemcpy(table)");
        if (rc) { (void)hipFree(blob); return rc; }
    }
    int32_t *ibase = (int32_t *)((char *)blob + dbytes);
    if (!ints.empty()) {
        rc = vk::hip_check(hipMemcpy(ibase, ints.data(), ints.size() * sizeof(int32_t),
                                     hipMemcpyHostToDevice), "hipMemcpy(table)");
        if (rc) { (void)hipFree(blob); return rc; }
    }
    vk_table *t = new vk_table();
    t->blob = blob;
    t->n_sets = d->n_sets; t->n_members = d->n_members; t->n_upd = d->n_upd; t->n_exch = d->n_exch;
    t->n_ib = (int32_t)ints.size(); t->n_db = (int32_t)dbl.size();
    vk_dev_table &v = t->dev;
    v.ib = ibase;
    v.db = (const double *)blob;
    v.n_species = d->n_species; v.n_dyn = d->n_dyn; v.n_reactions = d->n_reactions;
    v.n_rate_laws = L; v.n_params = d->n_params; v.n_ext = d->n_ext;
    v.o_upd_coeff = 0;
    v.o_ex_coeff = d->n_upd;
    v.o_rl_reaction = (int32_t)segs[0].off; v.o_rl_enzyme = (int32_t)segs[1].off;
    v.o_rl_kcat = (int32_t)segs[2].off; v.o_rl_num_ptr = (int32_t)segs[3].off;
    v.o_rl_den_ptr = (int32_t)segs[4].off; v.o_set_ptr = (int32_t)segs[5].off;
    v.o_mem_species = (int32_t)segs[6].off; v.o_mem_param = (int32_t)segs[7].off;
    v.o_upd_ptr = (int32_t)segs[8].off; v.o_upd_rxn = (int32_t)segs[9].off;
    v.o_ex_ptr = (int32_t)segs[10].off; v.o_ex_rxn = (int32_t)segs[11].off;
    v.o_rx_ptr = (int32_t)segs[12].off; v.o_rx_rl = (int32_t)segs[13].off;
    *out = t;
    return VK_OK;
}

extern "C" int vk_table_destroy(vk_table *t) {
    if (!t) return VK_OK;
    if (t->spec_module) (void)hipModuleUnload(t->spec_module);
    int rc = vk::hip_check(hipFree(t->blob), "hipFree(table)");
    delete t;
    return rc;
}

// Compile a network-specialised integrator (source generated from this same
// table by lens_amd/codegen.py) with hiprtc for gfx950 and attach it.
extern "C" int vk_table_specialize(vk_table *t, const char *source) {
    if (!t || !source) {
        vk::set_error("vk_table_specialize: null argument");
        return VK_ERR_ARG;
    }
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, source, "vk_dopri5_spec.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) {
        vk::set_error("vk_table_specialize: hiprtcCreateProgram failed");
        return VK_ERR_HIP;
    }
    const char *opts[] = {"--offload-arch=gfx950", "-O3", "-ffp-contract=off", "-std=c++17"};
    hiprtcResult cr = hiprtcCompileProgram(prog, 4, opts);
    if (cr != HIPRTC_SUCCESS) {
        size_t log_size = 0;
        hiprtcGetProgramLogSize(prog, &log_size);
        std::vector<char> log(log_size + 1, 0);
        if (log_size) hiprtcGetProgramLog(prog, log.data());
        vk::set_error("vk_table_specialize: compile failed: %.400s", log.data());
        hiprtcDestroyProgram(&prog);
        return VK_ERR_HIP;
    }
    size_t code_size = 0;
    hiprtcGetCodeSize(prog, &code_size);
    std::vector<char> code(code_size);
    hiprtcGetCode(prog, code.data());
    hiprtcDestroyProgram(&prog);
    hipModule_t mod;
    int rc = vk::hip_check(hipModuleLoadData(&mod, code.data()), "hipModuleLoadData(spec)");
    if (rc) return rc;
    // the source defines the agent-per-lane kernel, the agent-per-wavefront one, or both
    hipFunction_t fn = nullptr, fw = nullptr, fm = nullptr, fg = nullptr;
    if (hipModuleGetFunction(&fn, mod, "vk_dopri5_spec") != hipSuccess) fn = nullptr;
    if (hipModuleGetFunction(&fg, mod, "vk_dopri5_spec_gather") != hipSuccess) fg = nullptr;
    if (hipModuleGetFunction(&fw, mod, "vk_dopri5_wspec") != hipSuccess) fw = nullptr;
    if (hipModuleGetFunction(&fm, mod, "vk_dopri5_spec_multi") != hipSuccess) fm = nullptr;
    (void)hipGetLastError();
    if (!fn && !fw) {
        (void)hipModuleUnload(mod);
        vk::set_error("vk_table_specialize: the source defines neither vk_dopri5_spec nor vk_dopri5_wspec");
        return VK_ERR_ARG;
    }
    if (t->spec_module) (void)hipModuleUnload(t->spec_module);
    t->spec_module = mod;
    t->spec_dopri5 = fn;
    t->spec_wave = fw;
    t->spec_wave_waves = 4;
    if (fw) {   // the template's __launch_bounds__(64 * DW_WAVES) says how many agents a workgroup takes
        int mt = 0;
        if (hipFuncGetAttribute(&mt, HIP_FUNC_ATTRIBUTE_MAX_THREADS_PER_BLOCK, fw) == hipSuccess && mt >= 64 &&
            mt % 64 == 0)
            t->spec_wave_waves = mt / 64;
        (void)hipGetLastError();
    }
    t->spec_multi = fm;
    t->spec_gather = fg;
    return VK_OK;
}

// ---------------------------------------------------------------------------
// exact (reference-order) rate law, species/params read from global SoA
// ---------------------------------------------------------------------------

// cofactor_numerator / cofactor_denominator (kinetic_rate_laws.py:100-104):
// a falsy Km (0, -0) gives 0 in the numerator and 1 in the denominator.
__device__ __forceinline__ double rate_law_exact(const vk_dev_table &t, int l,
                                                 const double *__restrict__ params,
                                                 const double *__restrict__ conc, int64_t ld,
                                                 int64_t a) {
    double num = 0.0;
    const int ns0 = TI(t, rl_num_ptr, l), ns1 = TI(t, rl_num_ptr, l + 1);
    for (int s = ns0; s < ns1; ++s) {
        double term = 1.0;
        const int m0 = TI(t, set_ptr, s), m1 = TI(t, set_ptr, s + 1);
        for (int m = m0; m < m1; ++m) {
            const double km = params[(int64_t)TI(t, mem_param, m) * ld + a];
            const double c = conc[(int64_t)TI(t, mem_species, m) * ld + a];
            term = term * (km != 0.0 ? c / km : 0.0);
        }
        num = num + params[(int64_t)TI(t, rl_kcat, l) * ld + a] * term;
    }
    num = num * conc[(int64_t)TI(t, rl_enzyme, l) * ld + a];
    double den = 1.0;
    const int ds0 = TI(t, rl_den_ptr, l), ds1 = TI(t, rl_den_ptr, l + 1);
    for (int s = ds0; s < ds1; ++s) {
        double term = 1.0;
        const int m0 = TI(t, set_ptr, s), m1 = TI(t, set_ptr, s + 1);
        for (int m = m0; m < m1; ++m) {
            const double km = params[(int64_t)TI(t, mem_param, m) * ld + a];
            const double c = conc[(int64_t)TI(t, mem_species, m) * ld + a];
            term = term * (km != 0.0 ? 1.0 + c / km : 1.0);
        }
        den = den + (term - 1.0);
    }
    return num / den;
}

__device__ __forceinline__ void fluxes_exact(const vk_dev_table &t, const double *__restrict__ params,
                                             const double *__restrict__ conc, double *__restrict__ flux,
                                             int64_t ld, int64_t a) {
    for (int r = 0; r < t.n_reactions; ++r) flux[(int64_t)r * ld + a] = 0.0;
    for (int l = 0; l < t.n_rate_laws; ++l) {
        const double v = rate_law_exact(t, l, params, conc, ld, a);
        const int64_t idx = (int64_t)TI(t, rl_reaction, l) * ld + a;
        flux[idx] = flux[idx] + v;
    }
}

// Python int(x) truncates toward zero; out-of-range / non-finite -> flagged.
__device__ __forceinline__ int64_t trunc_count(double x, int32_t &st) {
    if (!(fabs(x) < 9.2e18)) {
        st |= VK_AGENT_NONFINITE;
        return 0;
    }
    return (int64_t)x;
}

__global__ __launch_bounds__(256) void k_rate_fluxes(vk_dev_table t, int64_t n, int64_t ld,
                                                     const double *__restrict__ params,
                                                     const double *__restrict__ conc,
                                                     double *__restrict__ flux) {
    const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= n) return;
    fluxes_exact(t, params, conc, flux, ld, a);
}

// ConvenienceKinetics.next_update (convenience_kinetics.py:320-349) + the
// accumulate updater: conc_s += (0 + sum_j (coeff_j*flux)*dt), counts_e =
// sum_j int(((coeff_j*flux)*dt)*m2c).
__global__ __launch_bounds__(256) void k_step_euler(vk_dev_table t, int64_t n, int64_t ld, double dt,
                                                    const double *__restrict__ params,
                                                    double *__restrict__ conc,
                                                    const double *__restrict__ m2c,
                                                    double *__restrict__ delta,
                                                    double *__restrict__ flux,
                                                    int64_t *__restrict__ counts,
                                                    int32_t *__restrict__ status) {
    const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= n) return;
    fluxes_exact(t, params, conc, flux, ld, a);
    int32_t st = 0;
    for (int s = 0; s < t.n_dyn; ++s) {
        double d = 0.0;
        const int j0 = TI(t, upd_ptr, s), j1 = TI(t, upd_ptr, s + 1);
        for (int j = j0; j < j1; ++j)
            d = d + (TD(t, upd_coeff, j) * flux[(int64_t)TI(t, upd_rxn, j) * ld + a]) * dt;
        const int64_t idx = (int64_t)s * ld + a;
        if (delta) {
            if (!isfinite(d)) st |= VK_AGENT_NONFINITE;
            delta[idx] = d;
        } else {
            const double v = conc[idx] + d;
            if (!isfinite(v)) st |= VK_AGENT_NONFINITE;
            conc[idx] = v;
        }
    }
    const double mc = m2c[a];
    for (int e = 0; e < t.n_ext; ++e) {
        int64_t c = 0;
        const int j0 = TI(t, ex_ptr, e), j1 = TI(t, ex_ptr, e + 1);
        for (int j = j0; j < j1; ++j) {
            const double sf = (TD(t, ex_coeff, j) * flux[(int64_t)TI(t, ex_rxn, j) * ld + a]) * dt;
            c += trunc_count(sf * mc, st);
        }
        counts[(int64_t)e * ld + a] = c;
    }
    if (status) status[a] = st;
}

static int check_agents(const char *fn, const vk_table *t, int64_t n, int64_t ld) {
    if (!t) {
        vk::set_error("%s: null table", fn);
        return VK_ERR_ARG;
    }
    if (n < 0 || ld < n) {
        vk::set_error("%s: need 0 <= n_agents <= ld (n=%lld ld=%lld)", fn, (long long)n, (long long)ld);
        return VK_ERR_ARG;
    }
    return VK_OK;
}

extern "C" int vk_rate_fluxes(const vk_table *t, int64_t n, int64_t ld, const double *params,
                              const double *conc, double *flux, vk_stream_t stream) {
    int rc = check_agents("vk_rate_fluxes", t, n, ld);
    if (rc || n == 0) return rc;
    if (!params || !conc || !flux) {
        vk::set_error("vk_rate_fluxes: null array");
        return VK_ERR_ARG;
    }
    const unsigned blocks = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(k_rate_fluxes, dim3(blocks), dim3(256), 0, (hipStream_t)stream, t->dev, n, ld,
                       params, conc, flux);
    return vk::launch_check("k_rate_fluxes");
}

extern "C" int vk_step_euler(const vk_table *t, int64_t n, int64_t ld, double dt, const double *params,
                             double *conc, const double *m2c, double *delta, double *flux, int64_t *counts,
                             int32_t *status, vk_stream_t stream) {
    int rc = check_agents("vk_step_euler", t, n, ld);
    if (rc || n == 0) return rc;
    if (!params || !conc || !m2c || !flux || (!counts && t->dev.n_ext > 0)) {
        vk::set_error("vk_step_euler: null array");
        return VK_ERR_ARG;
    }
    const unsigned blocks = (unsigned)((n + 255) / 256);
    hipLaunchKernelGGL(k_step_euler, dim3(blocks), dim3(256), 0, (hipStream_t)stream, t->dev, n, ld, dt,
                       params, conc, m2c, delta, flux, counts, status);
    return vk::launch_check("k_step_euler");
}

// ---------------------------------------------------------------------------
// Dormand-Prince 5(4), agent per lane
// ---------------------------------------------------------------------------
//
// y = [dyn species (n_dyn) | per-reaction flux integrals (n_reactions)], NY
// entries, a compile-time constant so the seven stage vectors live in VGPRs.
// LDS tile (BS lanes): rows [0,n_species) species, then n_reactions flux
// rows, then n_params parameter rows holding kcat or 1/Km (0 for a falsy Km).

namespace dp {
constexpr double a21 = 1.0 / 5.0;
constexpr double a31 = 3.0 / 40.0, a32 = 9.0 / 40.0;
constexpr double a41 = 44.0 / 45.0, a42 = -56.0 / 15.0, a43 = 32.0 / 9.0;
constexpr double a51 = 19372.0 / 6561.0, a52 = -25360.0 / 2187.0, a53 = 64448.0 / 6561.0,
                 a54 = -212.0 / 729.0;
constexpr double a61 = 9017.0 / 3168.0, a62 = -355.0 / 33.0, a63 = 46732.0 / 5247.0,
                 a64 = 49.0 / 176.0, a65 = -5103.0 / 18656.0;
constexpr double b1 = 35.0 / 384.0, b3 = 500.0 / 1113.0, b4 = 125.0 / 192.0,
                 b5 = -2187.0 / 6784.0, b6 = 11.0 / 84.0;
// e = b - bhat (4th-order embedded), scipy RK45's E up to sign
constexpr double e1 = 71.0 / 57600.0, e3 = -71.0 / 16695.0, e4 = 71.0 / 1920.0,
                 e5 = -17253.0 / 339200.0, e6 = 22.0 / 525.0, e7 = -1.0 / 40.0;
constexpr double SAFETY = 0.9, MIN_FACTOR = 0.2, MAX_FACTOR = 10.0;

// The adaptive kernels are tolerance-parity (within 1e-6 of odeint, SURVEY
// 8a), not bit-parity, so they use the cheap forms of their two costliest
// operations; the specialised kernel (vk_dopri5_spec.hip.in) uses the same
// two, so it stays bit-identical to the table walk.
// a/b by the hardware reciprocal plus one Newton step (~1e-15 relative, as
// vk_kremling.hip's; a second step bought nothing the 1e-6 odeint bar sees;
// a zero divisor gives NaN instead of inf -- flagged non-finite either way).
__device__ __forceinline__ double fdiv(double a, double b) {
    double r = __builtin_amdgcn_rcp(b);
    r = fma(fma(-b, r, 1.0), r, r);
    return a * r;
}

// en^-0.2 for the step-size factor (scipy RK45's error_norm ** (-1/5)) without
// libm's exp2 / log2: a single-precision estimate from the hardware v_log_f32 /
// v_exp_f32 (~1e-6 relative), then two Newton steps on en * y^5 = 1 in double
// (quadratic: ~1e-11, then rounding).  en is clamped to [1e-30, 1e30] so the
// float stays normal; outside that range the factor is capped anyway (at 10
// for en < 1e-30, at 0.2 for en > 1e30, callers' fmin / fmax).  The same code in
// every DP45 kernel (vk_kinetics.hip, the specialised templates, vk_kremling.hip)
// keeps them bit-identical to one another.  exp2(log2()) kept its polynomial
// constants in VGPRs across the attempt loop: the C5 wavefront kernel spilled
// them and reloaded eight in series per attempt (round 6).
__device__ __forceinline__ double step_pow(double en) {
    const double e = fmin(fmax(en, 1e-30), 1e30);
    double y = (double)__builtin_amdgcn_exp2f(-0.2f * __builtin_amdgcn_logf((float)e));
#pragma unroll
    for (int it = 0; it < 2; ++it) {
        const double y2 = y * y;
        const double r = fma(-e, y2 * y2 * y, 1.0);   // 1 - e y^5
        y = fma(0.2 * y, r, y);
    }
    return y;
}
}  // namespace dp

constexpr int DP_BS = 256;

// One rate law from the LDS tile (1/Km precomputed): num*E/den.
__device__ __forceinline__ double rate_law_tile(const vk_dev_table &t, int l, const double *cl,
                                                const double *pl, int lane) {
    double num = 0.0;
    const int ns0 = TI(t, rl_num_ptr, l), ns1 = TI(t, rl_num_ptr, l + 1);
    for (int s = ns0; s < ns1; ++s) {
        double term = pl[TI(t, rl_kcat, l) * DP_BS + lane];
        const int m0 = TI(t, set_ptr, s), m1 = TI(t, set_ptr, s + 1);
        for (int m = m0; m < m1; ++m)
            term *= cl[TI(t, mem_species, m) * DP_BS + lane] * pl[TI(t, mem_param, m) * DP_BS + lane];
        num += term;
    }
    num *= cl[TI(t, rl_enzyme, l) * DP_BS + lane];
    double den = 1.0;
    const int ds0 = TI(t, rl_den_ptr, l), ds1 = TI(t, rl_den_ptr, l + 1);
    for (int s = ds0; s < ds1; ++s) {
        double term = 1.0;
        const int m0 = TI(t, set_ptr, s), m1 = TI(t, set_ptr, s + 1);
        for (int m = m0; m < m1; ++m)
            term *= fma(cl[TI(t, mem_species, m) * DP_BS + lane], pl[TI(t, mem_param, m) * DP_BS + lane], 1.0);
        den += term - 1.0;
    }
    return dp::fdiv(num, den);
}

template <int NY>
__device__ __forceinline__ void rhs_tile(const vk_dev_table &t, const double (&y)[NY], double (&dy)[NY],
                                         double *cl, double *fl, const double *pl, int lane) {
    const int nd = t.n_dyn;
#pragma unroll
    for (int i = 0; i < NY; ++i)
        if (i < nd) cl[i * DP_BS + lane] = y[i];
    for (int r = 0; r < t.n_reactions; ++r) fl[r * DP_BS + lane] = 0.0;
    for (int l = 0; l < t.n_rate_laws; ++l) {
        const double v = rate_law_tile(t, l, cl, pl, lane);
        const int r = TI(t, rl_reaction, l);
        fl[r * DP_BS + lane] += v;
    }
#pragma unroll
    for (int i = 0; i < NY; ++i) {
        if (i < nd) {
            double d = 0.0;
            const int j0 = TI(t, upd_ptr, i), j1 = TI(t, upd_ptr, i + 1);
            for (int j = j0; j < j1; ++j) d = fma(TD(t, upd_coeff, j), fl[TI(t, upd_rxn, j) * DP_BS + lane], d);
            dy[i] = d;
        } else if (i < nd + t.n_reactions) {
            dy[i] = fl[(i - nd) * DP_BS + lane];
        } else {
            dy[i] = 0.0;   // padding of the NY bucket
        }
    }
}

// RMS over the ny live components (entries >= ny pad the NY bucket)
template <int NY>
__device__ __forceinline__ double rms_norm(const double (&v)[NY], const double (&scale)[NY], int ny) {
    double s = 0.0;
#pragma unroll
    for (int i = 0; i < NY; ++i) {
        if (i < ny) {
            const double q = v[i] / scale[i];
            s = fma(q, q, s);
        }
    }
    return sqrt(s / ny);
}

template <int NY>
__global__ __launch_bounds__(DP_BS) void k_dopri5_thread(vk_dev_table t, int64_t n, int64_t ld, double dt,
                                                         double rtol, double atol, int max_steps,
                                                         const double *__restrict__ params,
                                                         double *__restrict__ conc,
                                                         const double *__restrict__ m2c,
                                                         double *__restrict__ delta,
                                                         double *__restrict__ h_state,
                                                         double *__restrict__ flux,
                                                         int64_t *__restrict__ counts,
                                                         int32_t *__restrict__ status,
                                                         int32_t *__restrict__ nsteps_out) {
    extern __shared__ double lds[];
    const int lane = threadIdx.x;
    const int64_t a = (int64_t)blockIdx.x * DP_BS + lane;
    double *cl = lds;                                 // [n_species][BS]
    double *fl = lds + t.n_species * DP_BS;           // [n_reactions][BS]
    double *pl = fl + t.n_reactions * DP_BS;          // [n_params][BS]
    if (a >= n) return;                               // no block-wide sync below

    // stage per-lane constants into the tile
    for (int s = t.n_dyn; s < t.n_species; ++s) cl[s * DP_BS + lane] = conc[(int64_t)s * ld + a];
    for (int p = 0; p < t.n_params; ++p) pl[p * DP_BS + lane] = params[(int64_t)p * ld + a];
    for (int m = 0; m < TI(t, set_ptr, TI(t, rl_den_ptr, t.n_rate_laws)); ++m) {
        const int p = TI(t, mem_param, m);
        const double km = params[(int64_t)p * ld + a];
        pl[p * DP_BS + lane] = (km != 0.0) ? 1.0 / km : 0.0;
    }

    const int nd = t.n_dyn;
    const int ny = nd + t.n_reactions;
    double y[NY], k1[NY], k2[NY], k3[NY], k4[NY], k5[NY], k6[NY], k7[NY], yt[NY];
#pragma unroll
    for (int i = 0; i < NY; ++i) y[i] = (i < nd) ? conc[(int64_t)i * ld + a] : 0.0;

    rhs_tile<NY>(t, y, k1, cl, fl, pl, lane);
    int32_t st = 0;
    double h = h_state ? h_state[a] : 0.0;
    if (!(h > 0.0)) {
        // scipy select_initial_step (order 4)
        double sc[NY];
#pragma unroll
        for (int i = 0; i < NY; ++i) sc[i] = fma(fabs(y[i]), rtol, atol);
        const double d0 = rms_norm<NY>(y, sc, ny), d1 = rms_norm<NY>(k1, sc, ny);
        double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
        h0 = fmin(h0, dt);
#pragma unroll
        for (int i = 0; i < NY; ++i) yt[i] = fma(h0, k1[i], y[i]);
        rhs_tile<NY>(t, yt, k2, cl, fl, pl, lane);
#pragma unroll
        for (int i = 0; i < NY; ++i) k2[i] = k2[i] - k1[i];
        const double d2 = rms_norm<NY>(k2, sc, ny) / h0;
        const double h1 = (d1 <= 1e-15 && d2 <= 1e-15) ? fmax(1e-6, h0 * 1e-3)
                                                        : pow(0.01 / fmax(d1, d2), 0.2);
        h = fmin(fmin(100.0 * h0, h1), dt);
    }

    double tt = 0.0;
    int ns = 0;
    bool rejected = false;
    double h_keep = h;
    while (tt < dt) {
        if (ns >= max_steps) { st |= VK_AGENT_MAX_STEPS; break; }
        if (h < 1e-14 * dt) { st |= VK_AGENT_H_UNDERFLOW; break; }
        double hs = h;
        bool last = false;
        if (tt + hs >= dt) { hs = dt - tt; last = true; }
        ++ns;
#pragma unroll
        for (int i = 0; i < NY; ++i) yt[i] = fma(hs, dp::a21 * k1[i], y[i]);
        rhs_tile<NY>(t, yt, k2, cl, fl, pl, lane);
#pragma unroll
        for (int i = 0; i < NY; ++i) yt[i] = fma(hs, fma(dp::a32, k2[i], dp::a31 * k1[i]), y[i]);
        rhs_tile<NY>(t, yt, k3, cl, fl, pl, lane);
#pragma unroll
        for (int i = 0; i < NY; ++i)
            yt[i] = fma(hs, fma(dp::a43, k3[i], fma(dp::a42, k2[i], dp::a41 * k1[i])), y[i]);
        rhs_tile<NY>(t, yt, k4, cl, fl, pl, lane);
#pragma unroll
        for (int i = 0; i < NY; ++i)
            yt[i] = fma(hs, fma(dp::a54, k4[i], fma(dp::a53, k3[i], fma(dp::a52, k2[i], dp::a51 * k1[i]))), y[i]);
        rhs_tile<NY>(t, yt, k5, cl, fl, pl, lane);
#pragma unroll
        for (int i = 0; i < NY; ++i)
            yt[i] = fma(hs, fma(dp::a65, k5[i], fma(dp::a64, k4[i], fma(dp::a63, k3[i],
                        fma(dp::a62, k2[i], dp::a61 * k1[i])))), y[i]);
        rhs_tile<NY>(t, yt, k6, cl, fl, pl, lane);
#pragma unroll
        for (int i = 0; i < NY; ++i)
            yt[i] = fma(hs, fma(dp::b6, k6[i], fma(dp::b5, k5[i], fma(dp::b4, k4[i],
                        fma(dp::b3, k3[i], dp::b1 * k1[i])))), y[i]);
        rhs_tile<NY>(t, yt, k7, cl, fl, pl, lane);
        double en = 0.0;
#pragma unroll
        for (int i = 0; i < NY; ++i) {
            if (i < ny) {
                const double err = hs * fma(dp::e7, k7[i], fma(dp::e6, k6[i], fma(dp::e5, k5[i],
                                       fma(dp::e4, k4[i], fma(dp::e3, k3[i], dp::e1 * k1[i])))));
                const double q = dp::fdiv(err, fma(fmax(fabs(y[i]), fabs(yt[i])), rtol, atol));
                en = fma(q, q, en);
            }
        }
        en = sqrt(en / ny);
        if (!isfinite(en)) { st |= VK_AGENT_NONFINITE; break; }
        if (en < 1.0) {
            double factor = (en == 0.0) ? dp::MAX_FACTOR : fmin(dp::MAX_FACTOR, dp::SAFETY * dp::step_pow(en));
            if (rejected) factor = fmin(1.0, factor);
            tt = last ? dt : tt + hs;
#pragma unroll
            for (int i = 0; i < NY; ++i) { y[i] = yt[i]; k1[i] = k7[i]; }
            h_keep = last ? fmax(h, hs * factor) : hs * factor;
            h = hs * factor;
            rejected = false;
        } else {
            h = hs * fmax(dp::MIN_FACTOR, dp::SAFETY * dp::step_pow(en));
            rejected = true;
        }
    }

    // write back: species, mean fluxes, exchange counts from the integrals
#pragma unroll
    for (int i = 0; i < NY; ++i) {
        if (i < nd) {
            if (!isfinite(y[i])) st |= VK_AGENT_NONFINITE;
            const int64_t idx = (int64_t)i * ld + a;
            if (delta)
                delta[idx] = y[i] - conc[idx];
            else
                conc[idx] = y[i];
        } else if (i < ny) {
            fl[(i - nd) * DP_BS + lane] = y[i];      // integrals back into the tile
            flux[(int64_t)(i - nd) * ld + a] = y[i] / dt;
        }
    }
    const double mc = m2c[a];
    for (int e = 0; e < t.n_ext; ++e) {
        int64_t c = 0;
        const int j0 = TI(t, ex_ptr, e), j1 = TI(t, ex_ptr, e + 1);
        for (int j = j0; j < j1; ++j)
            c += trunc_count((TD(t, ex_coeff, j) * fl[TI(t, ex_rxn, j) * DP_BS + lane]) * mc, st);
        counts[(int64_t)e * ld + a] = c;
    }
    if (h_state) h_state[a] = h_keep;
    if (status) status[a] = st;
    if (nsteps_out) nsteps_out[a] = ns;
}

// ---------------------------------------------------------------------------
// Dormand-Prince 5(4), agent per WAVEFRONT (networks too large for a lane)
// ---------------------------------------------------------------------------
//
// One 64-lane wavefront integrates one agent; a workgroup of 4 waves stages
// the (shared, read-only) rate-law table into LDS once, then each wave runs its
// own agent with wave-local synchronisation only (waves take different numbers
// of steps, so no block barrier after staging).  Component i of y = [dyn species |
// flux integrals] lives in lane i % 64, slot i / 64 (NSLOT slots per lane).
// Each RHS: lanes publish their species to the agent's LDS tile, lane l
// evaluates rate laws l, l+64, ... (same arithmetic as rate_law_tile), lane r
// sums reaction r's rate laws in evaluation order, lanes form dy for their
// components.  The RMS error norm is a wavefront sum (DPP/shuffle butterfly),
// so step acceptance, h and t are wave-uniform: no divergence at all.
// Results agree with the lane kernels to rounding (only the order of the
// norm's sum differs: a pairwise tree here, a running sum there).

constexpr int DW = 64;
constexpr int DW_WAVES = 4;   // agents (waves) per workgroup

// LDS communication between the lanes of ONE wave: a wave's LDS operations
// execute in order, so only the compiler must be kept from reordering.
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Wavefront sum, identical in every lane: a butterfly from the smallest
// distance up.  Distances 1 and 2 are quad_perm DPP moves; once quads (then
// 8-lane groups) hold equal values, row_half_mirror / row_mirror pair them
// exactly as distances 4 / 8 would; distances 16 and 32 use the gfx950 row
// swaps (v_permlane16/32_swap), after which each lane holds v[l] and
// v[l ^ d] and adds them (FP addition commutes, so every lane gets the same
// bits).  No LDS round trip, unlike __shfl_xor (ds_bpermute).
__device__ __forceinline__ double dpp_pair(double v, int ctrl) {
    int2 x = __builtin_bit_cast(int2, v);
    int2 y;
    switch (ctrl) {   // the DPP control must be a compile-time constant
        case 0xB1:
            y.x = __builtin_amdgcn_mov_dpp(x.x, 0xB1, 0xf, 0xf, false);
            y.y = __builtin_amdgcn_mov_dpp(x.y, 0xB1, 0xf, 0xf, false);
            break;
        case 0x4E:
            y.x = __builtin_amdgcn_mov_dpp(x.x, 0x4E, 0xf, 0xf, false);
            y.y = __builtin_amdgcn_mov_dpp(x.y, 0x4E, 0xf, 0xf, false);
            break;
        case 0x141:
            y.x = __builtin_amdgcn_mov_dpp(x.x, 0x141, 0xf, 0xf, false);
            y.y = __builtin_amdgcn_mov_dpp(x.y, 0x141, 0xf, 0xf, false);
            break;
        default:
            y.x = __builtin_amdgcn_mov_dpp(x.x, 0x140, 0xf, 0xf, false);
            y.y = __builtin_amdgcn_mov_dpp(x.y, 0x140, 0xf, 0xf, false);
            break;
    }
    return v + __builtin_bit_cast(double, y);
}

__device__ __forceinline__ double wave_sum(double v) {
    v = dpp_pair(v, 0xB1);    // quad_perm [1,0,3,2]: lane ^ 1
    v = dpp_pair(v, 0x4E);    // quad_perm [2,3,0,1]: lane ^ 2
    v = dpp_pair(v, 0x141);   // row_half_mirror: the other quad of the 8-lane group
    v = dpp_pair(v, 0x140);   // row_mirror: the other 8-lane group of the row
    int2 x = __builtin_bit_cast(int2, v);
    auto lo = __builtin_amdgcn_permlane16_swap(x.x, x.x, false, false);
    auto hi = __builtin_amdgcn_permlane16_swap(x.y, x.y, false, false);
    v = __builtin_bit_cast(double, make_int2(lo[0], hi[0])) + __builtin_bit_cast(double, make_int2(lo[1], hi[1]));
    x = __builtin_bit_cast(int2, v);
    lo = __builtin_amdgcn_permlane32_swap(x.x, x.x, false, false);
    hi = __builtin_amdgcn_permlane32_swap(x.y, x.y, false, false);
    return __builtin_bit_cast(double, make_int2(lo[0], hi[0])) + __builtin_bit_cast(double, make_int2(lo[1], hi[1]));
}

// rate law l from the agent's LDS tile (cl: species, pl: kcat or 1/Km);
// table indices are lane-divergent here, so they are plain (vector) loads
__device__ __forceinline__ double rate_law_wave(const vk_dev_table &t, const int32_t *ib, int l, const double *cl,
                                                const double *pl) {
    double num = 0.0;
    const int ns0 = ib[t.o_rl_num_ptr + l], ns1 = ib[t.o_rl_num_ptr + l + 1];
    const double kcat = pl[ib[t.o_rl_kcat + l]];
    for (int s = ns0; s < ns1; ++s) {
        double term = kcat;
        const int m0 = ib[t.o_set_ptr + s], m1 = ib[t.o_set_ptr + s + 1];
        for (int m = m0; m < m1; ++m) term *= cl[ib[t.o_mem_species + m]] * pl[ib[t.o_mem_param + m]];
        num += term;
    }
    num *= cl[ib[t.o_rl_enzyme + l]];
    double den = 1.0;
    const int ds0 = ib[t.o_rl_den_ptr + l], ds1 = ib[t.o_rl_den_ptr + l + 1];
    for (int s = ds0; s < ds1; ++s) {
        double term = 1.0;
        const int m0 = ib[t.o_set_ptr + s], m1 = ib[t.o_set_ptr + s + 1];
        for (int m = m0; m < m1; ++m) term *= fma(cl[ib[t.o_mem_species + m]], pl[ib[t.o_mem_param + m]], 1.0);
        den += term - 1.0;
    }
    return dp::fdiv(num, den);
}

template <int NSLOT>
__device__ __forceinline__ void rhs_wave(const vk_dev_table &t, const int32_t *ib, const double *db,
                                         const double (&y)[NSLOT], double (&dy)[NSLOT], double *cl, double *fl,
                                         const double *pl, double *rl, int lane) {
    const int nd = t.n_dyn, nr = t.n_reactions, nl = t.n_rate_laws;
#pragma unroll
    for (int k = 0; k < NSLOT; ++k) {
        const int i = lane + DW * k;
        if (i < nd) cl[i] = y[k];
    }
    wave_sync();
    for (int l = lane; l < nl; l += DW) rl[l] = rate_law_wave(t, ib, l, cl, pl);
    wave_sync();
    for (int r = lane; r < nr; r += DW) {
        double f = 0.0;
        for (int k = ib[t.o_rx_ptr + r]; k < ib[t.o_rx_ptr + r + 1]; ++k) f += rl[ib[t.o_rx_rl + k]];
        fl[r] = f;
    }
    wave_sync();
#pragma unroll
    for (int k = 0; k < NSLOT; ++k) {
        const int i = lane + DW * k;
        double d = 0.0;
        if (i < nd) {
            for (int j = ib[t.o_upd_ptr + i]; j < ib[t.o_upd_ptr + i + 1]; ++j)
                d = fma(db[t.o_upd_coeff + j], fl[ib[t.o_upd_rxn + j]], d);
        } else if (i < nd + nr) {
            d = fl[i - nd];
        }
        dy[k] = d;
    }
    wave_sync();   // the next RHS overwrites cl / fl
}

template <int NSLOT>
__device__ __forceinline__ double wave_rms(const double (&v)[NSLOT], const double (&sc)[NSLOT], int lane, int ny) {
    double s = 0.0;
#pragma unroll
    for (int k = 0; k < NSLOT; ++k) {
        if (lane + DW * k < ny) {
            const double q = v[k] / sc[k];
            s = fma(q, q, s);
        }
    }
    return sqrt(wave_sum(s) / ny);
}

template <int NSLOT>
__global__ __launch_bounds__(DW * DW_WAVES) void k_dopri5_wave(vk_dev_table t, int n_ib, int n_db, int tile,
                                                               int64_t n, int64_t ld, double dt, double rtol,
                                                               double atol, int max_steps,
                                                               const double *__restrict__ params,
                                                               double *__restrict__ conc,
                                                               const double *__restrict__ m2c,
                                                               double *__restrict__ delta,
                                                               double *__restrict__ h_state,
                                                               double *__restrict__ flux,
                                                               int64_t *__restrict__ counts,
                                                               int32_t *__restrict__ status,
                                                               int32_t *__restrict__ nsteps_out) {
    extern __shared__ double lds[];
    // [table doubles | table ints | one agent tile per wave]
    double *db = lds;
    int32_t *ib = (int32_t *)(lds + n_db);
    for (int i = threadIdx.x; i < n_db; i += DW * DW_WAVES) db[i] = t.db[i];
    for (int i = threadIdx.x; i < n_ib; i += DW * DW_WAVES) ib[i] = t.ib[i];
    __syncthreads();   // the only block barrier: waves run independent agents from here on
    const int lane = threadIdx.x & (DW - 1), w = threadIdx.x / DW;
    const int64_t a = (int64_t)blockIdx.x * DW_WAVES + w;
    if (a >= n) return;
    const int ns_ = t.n_species, nr = t.n_reactions, np_ = t.n_params, nd = t.n_dyn;
    const int ny = nd + nr;
    double *cl = lds + n_db + (n_ib + 1) / 2 + (int64_t)w * tile;   // [n_species]
    double *fl = cl + ns_;            // [n_reactions]
    double *pl = fl + nr;             // [n_params]  kcat or 1/Km
    double *rl = pl + np_;            // [n_rate_laws]

    for (int s = lane; s < ns_; s += DW) cl[s] = conc[(int64_t)s * ld + a];
    for (int p = lane; p < np_; p += DW) pl[p] = params[(int64_t)p * ld + a];
    wave_sync();
    const int n_mem = ib[t.o_set_ptr + ib[t.o_rl_den_ptr + t.n_rate_laws]];
    for (int m = lane; m < n_mem; m += DW) {
        const int p = ib[t.o_mem_param + m];
        const double km = params[(int64_t)p * ld + a];
        pl[p] = (km != 0.0) ? 1.0 / km : 0.0;
    }
    wave_sync();

    double y[NSLOT], k1[NSLOT], k2[NSLOT], k3[NSLOT], k4[NSLOT], k5[NSLOT], k6[NSLOT], k7[NSLOT], yt[NSLOT];
#pragma unroll
    for (int k = 0; k < NSLOT; ++k) {
        const int i = lane + DW * k;
        y[k] = (i < nd) ? cl[i] : 0.0;
    }
    rhs_wave<NSLOT>(t, ib, db, y, k1, cl, fl, pl, rl, lane);
    int32_t st = 0;
    double h = h_state ? h_state[a] : 0.0;
    if (!(h > 0.0)) {   // scipy select_initial_step (order 4)
        double sc[NSLOT];
#pragma unroll
        for (int k = 0; k < NSLOT; ++k) sc[k] = fma(fabs(y[k]), rtol, atol);
        const double d0 = wave_rms<NSLOT>(y, sc, lane, ny), d1 = wave_rms<NSLOT>(k1, sc, lane, ny);
        double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
        h0 = fmin(h0, dt);
#pragma unroll
        for (int k = 0; k < NSLOT; ++k) yt[k] = fma(h0, k1[k], y[k]);
        rhs_wave<NSLOT>(t, ib, db, yt, k2, cl, fl, pl, rl, lane);
#pragma unroll
        for (int k = 0; k < NSLOT; ++k) k2[k] = k2[k] - k1[k];
        const double d2 = wave_rms<NSLOT>(k2, sc, lane, ny) / h0;
        const double h1 = (d1 <= 1e-15 && d2 <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : pow(0.01 / fmax(d1, d2), 0.2);
        h = fmin(fmin(100.0 * h0, h1), dt);
    }

    double tt = 0.0, h_keep = h;
    int nsteps = 0;
    bool rejected = false;
    while (tt < dt) {   // every quantity in the loop control is wave-uniform
        if (nsteps >= max_steps) { st |= VK_AGENT_MAX_STEPS; break; }
        if (h < 1e-14 * dt) { st |= VK_AGENT_H_UNDERFLOW; break; }
        double hs = h;
        bool last = false;
        if (tt + hs >= dt) { hs = dt - tt; last = true; }
        ++nsteps;
#pragma unroll
        for (int k = 0; k < NSLOT; ++k) yt[k] = fma(hs, dp::a21 * k1[k], y[k]);
        rhs_wave<NSLOT>(t, ib, db, yt, k2, cl, fl, pl, rl, lane);
#pragma unroll
        for (int k = 0; k < NSLOT; ++k) yt[k] = fma(hs, fma(dp::a32, k2[k], dp::a31 * k1[k]), y[k]);
        rhs_wave<NSLOT>(t, ib, db, yt, k3, cl, fl, pl, rl, lane);
#pragma unroll
        for (int k = 0; k < NSLOT; ++k)
            yt[k] = fma(hs, fma(dp::a43, k3[k], fma(dp::a42, k2[k], dp::a41 * k1[k])), y[k]);
        rhs_wave<NSLOT>(t, ib, db, yt, k4, cl, fl, pl, rl, lane);
#pragma unroll
        for (int k = 0; k < NSLOT; ++k)
            yt[k] = fma(hs, fma(dp::a54, k4[k], fma(dp::a53, k3[k], fma(dp::a52, k2[k], dp::a51 * k1[k]))), y[k]);
        rhs_wave<NSLOT>(t, ib, db, yt, k5, cl, fl, pl, rl, lane);
#pragma unroll
        for (int k = 0; k < NSLOT; ++k)
            yt[k] = fma(hs, fma(dp::a65, k5[k], fma(dp::a64, k4[k], fma(dp::a63, k3[k],
                        fma(dp::a62, k2[k], dp::a61 * k1[k])))), y[k]);
        rhs_wave<NSLOT>(t, ib, db, yt, k6, cl, fl, pl, rl, lane);
#pragma unroll
        for (int k = 0; k < NSLOT; ++k)
            yt[k] = fma(hs, fma(dp::b6, k6[k], fma(dp::b5, k5[k], fma(dp::b4, k4[k],
                        fma(dp::b3, k3[k], dp::b1 * k1[k])))), y[k]);
        rhs_wave<NSLOT>(t, ib, db, yt, k7, cl, fl, pl, rl, lane);
        double e2 = 0.0;
#pragma unroll
        for (int k = 0; k < NSLOT; ++k) {
            if (lane + DW * k < ny) {
                const double err = hs * fma(dp::e7, k7[k], fma(dp::e6, k6[k], fma(dp::e5, k5[k],
                                       fma(dp::e4, k4[k], fma(dp::e3, k3[k], dp::e1 * k1[k])))));
                const double q = dp::fdiv(err, fma(fmax(fabs(y[k]), fabs(yt[k])), rtol, atol));
                e2 = fma(q, q, e2);
            }
        }
        const double en = sqrt(wave_sum(e2) / ny);
        if (!isfinite(en)) { st |= VK_AGENT_NONFINITE; break; }
        if (en < 1.0) {
            double factor = (en == 0.0) ? dp::MAX_FACTOR : fmin(dp::MAX_FACTOR, dp::SAFETY * dp::step_pow(en));
            if (rejected) factor = fmin(1.0, factor);
            tt = last ? dt : tt + hs;
#pragma unroll
            for (int k = 0; k < NSLOT; ++k) { y[k] = yt[k]; k1[k] = k7[k]; }
            h_keep = last ? fmax(h, hs * factor) : hs * factor;
            h = hs * factor;
            rejected = false;
        } else {
            h = hs * fmax(dp::MIN_FACTOR, dp::SAFETY * dp::step_pow(en));
            rejected = true;
        }
    }

    // write back: species, mean fluxes; integrals -> LDS for the exchange counts
    bool bad = false;
#pragma unroll
    for (int k = 0; k < NSLOT; ++k) {
        const int i = lane + DW * k;
        if (i < nd) {
            bad |= !isfinite(y[k]);
            const int64_t idx = (int64_t)i * ld + a;
            if (delta)
                delta[idx] = y[k] - conc[idx];
            else
                conc[idx] = y[k];
        } else if (i < ny) {
            fl[i - nd] = y[k];
            flux[(int64_t)(i - nd) * ld + a] = y[k] / dt;
        }
    }
    wave_sync();
    if (__any(bad)) st |= VK_AGENT_NONFINITE;
    const double mc = m2c[a];
    int32_t cst = 0;
    for (int e = lane; e < t.n_ext; e += DW) {
        int64_t c = 0;
        for (int j = ib[t.o_ex_ptr + e]; j < ib[t.o_ex_ptr + e + 1]; ++j)
            c += trunc_count((db[t.o_ex_coeff + j] * fl[ib[t.o_ex_rxn + j]]) * mc, cst);
        counts[(int64_t)e * ld + a] = c;
    }
    if (__any(cst != 0)) st |= VK_AGENT_NONFINITE;
    if (lane == 0) {
        if (h_state) h_state[a] = h_keep;
        if (status) status[a] = st;
        if (nsteps_out) nsteps_out[a] = nsteps;
    }
}

template <int NSLOT>
static int launch_dopri5_wave(const vk_table *t, int64_t n, int64_t ld, double dt, const vk_ode_opts *o,
                              const double *params, double *conc, const double *m2c, double *delta,
                              double *h_state, double *flux, int64_t *counts, int32_t *status, int32_t *nsteps,
                              hipStream_t stream) {
    const vk_dev_table &d = t->dev;
    const int tile = d.n_species + d.n_reactions + d.n_params + d.n_rate_laws;   // doubles per agent
    const size_t lds = ((size_t)t->n_db + (t->n_ib + 1) / 2 + (size_t)DW_WAVES * tile) * sizeof(double);
    if (lds > 160 * 1024) {
        vk::set_error("vk_step_dopri5: network needs %zu B of LDS per workgroup (> 160 KiB)", lds);
        return VK_ERR_LIMIT;
    }
    if (n > 0x1fffffff) {
        vk::set_error("vk_step_dopri5: agent-per-wavefront grid limited to 2^29 agents");
        return VK_ERR_LIMIT;
    }
    auto kern = k_dopri5_wave<NSLOT>;
    if (lds > 64 * 1024)
        (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
    const unsigned blocks = (unsigned)((n + DW_WAVES - 1) / DW_WAVES);
    hipLaunchKernelGGL(kern, dim3(blocks), dim3(DW * DW_WAVES), lds, stream, d, t->n_ib, t->n_db, tile, n, ld, dt,
                       o->rtol, o->atol, o->max_steps, params, conc, m2c, delta, h_state, flux, counts, status,
                       nsteps);
    return vk::launch_check("k_dopri5_wave");
}

template <int NY>
static int launch_dopri5(const vk_table *t, int64_t n, int64_t ld, double dt, const vk_ode_opts *o,
                         const double *params, double *conc, const double *m2c, double *delta, double *h_state,
                         double *flux, int64_t *counts, int32_t *status, int32_t *nsteps,
                         hipStream_t stream) {
    const size_t lds = (size_t)(t->dev.n_species + t->dev.n_reactions + t->dev.n_params) * DP_BS * sizeof(double);
    if (lds > 160 * 1024) {
        vk::set_error("vk_step_dopri5: network needs %zu B of LDS per 256-agent tile (> 160 KiB); "
                      "use the agent-per-wavefront variant", lds);
        return VK_ERR_LIMIT;
    }
    static bool attr_set = false;
    if (lds > 64 * 1024 && !attr_set) {
        (void)hipFuncSetAttribute((const void *)k_dopri5_thread<NY>,
                                  hipFuncAttributeMaxDynamicSharedMemorySize, 160 * 1024);
        attr_set = true;
    }
    const unsigned blocks = (unsigned)((n + DP_BS - 1) / DP_BS);
    hipLaunchKernelGGL(k_dopri5_thread<NY>, dim3(blocks), dim3(DP_BS), lds, stream, t->dev, n, ld, dt, o->rtol,
                       o->atol, o->max_steps, params, conc, m2c, delta, h_state, flux, counts, status, nsteps);
    return vk::launch_check("k_dopri5_thread");
}

// n_steps agent-steps of dt per launch for agents that do not couple between
// One vk_step_dopri5 (variant 2) that also gathers the next step's local
// environment: after the integration, conc[map_row[i] * ld + a] := plane
// map_field[i] of `fields` at bin_lin[a], as vk_gather right after the kinetics.
// Threads per block of the agent-per-lane specialised kernels: 256, or 64 when
// the colony is small (fewer than 4 blocks of 256 per CU), so that its waves
// spread over every CU instead of 4 to a CU on a few CUs (C2: 157 waves).
static unsigned spec_threads(int64_t n) {
    static int cus = 0;
    if (cus == 0) {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
            hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0)
            cus = 256;
    }
    return n < (int64_t)256 * 4 * cus ? 64u : 256u;
}

extern "C" int vk_step_dopri5_gather(const vk_table *t, int64_t n, int64_t ld, double dt, const vk_ode_opts *o,
                                     const double *params, double *conc, const double *m2c, double *h_state,
                                     double *flux, int64_t *counts, int32_t *status, int32_t *nsteps,
                                     const double *fields, int64_t field_stride, const int32_t *bin_lin,
                                     const int32_t *map_field, const int32_t *map_row, int32_t n_map,
                                     vk_stream_t stream) {
    int rc = check_agents("vk_step_dopri5_gather", t, n, ld);
    if (rc || n == 0) return rc;
    if (!o || !params || !conc || !m2c || !flux || (!counts && t->dev.n_ext > 0) || n_map < 0 || n_map > 8 ||
        (n_map > 0 && (!fields || !bin_lin || !map_field || !map_row))) {
        vk::set_error("vk_step_dopri5_gather: null argument or n_map outside [0, 8]");
        return VK_ERR_ARG;
    }
    if (!(dt > 0.0) || !(o->rtol > 0.0) || !(o->atol >= 0.0) || o->max_steps <= 0) {
        vk::set_error("vk_step_dopri5_gather: need dt > 0, rtol > 0, atol >= 0, max_steps > 0");
        return VK_ERR_ARG;
    }
    if (!t->spec_gather) {
        vk::set_error("vk_step_dopri5_gather: needs vk_table_specialize with an agent-per-lane source first");
        return VK_ERR_ARG;
    }
    double rtol = o->rtol, atol = o->atol;
    int max_steps = o->max_steps, nm = n_map;
    void *args[] = {&n, &ld, &dt, &rtol, &atol, &max_steps, (void *)&params, &conc, (void *)&m2c, &h_state,
                    &flux, &counts, &status, &nsteps, (void *)&fields, &field_stride, (void *)&bin_lin,
                    (void *)&map_field, (void *)&map_row, &nm};
    const unsigned th = spec_threads(n), blocks = (unsigned)((n + th - 1) / th);
    return vk::hip_check(hipModuleLaunchKernel(t->spec_gather, blocks, 1, 1, th, 1, 1, 0, (hipStream_t)stream,
                                               args, nullptr),
                         "hipModuleLaunchKernel(vk_dopri5_spec_gather)");
}

// steps (held externals), with the network-specialised agent-per-lane kernel.
extern "C" int vk_step_dopri5_multi(const vk_table *t, int64_t n, int64_t ld, double dt, int32_t n_steps,
                                    const vk_ode_opts *o, const double *params, double *conc, const double *m2c,
                                    double *h_state, double *flux, int64_t step_flux, int64_t *counts,
                                    int64_t step_counts, int32_t *status, int32_t *nsteps, int64_t step_nsteps,
                                    vk_stream_t stream) {
    int rc = check_agents("vk_step_dopri5_multi", t, n, ld);
    if (rc || n == 0 || n_steps == 0) return rc;
    if (!o || !params || !conc || !m2c || !flux || (!counts && t->dev.n_ext > 0) || n_steps < 0) {
        vk::set_error("vk_step_dopri5_multi: null argument or negative step count");
        return VK_ERR_ARG;
    }
    if (!(dt > 0.0) || !(o->rtol > 0.0) || !(o->atol >= 0.0) || o->max_steps <= 0) {
        vk::set_error("vk_step_dopri5_multi: need dt > 0, rtol > 0, atol >= 0, max_steps > 0");
        return VK_ERR_ARG;
    }
    if (!t->spec_multi) {
        vk::set_error("vk_step_dopri5_multi: needs vk_table_specialize with an agent-per-lane source first");
        return VK_ERR_ARG;
    }
    if (n_steps > 1 && (step_flux < (int64_t)t->dev.n_reactions * ld || step_counts < (int64_t)t->dev.n_ext * ld ||
                        (nsteps && step_nsteps < ld))) {
        vk::set_error("vk_step_dopri5_multi: per-step output strides overlap");
        return VK_ERR_ARG;
    }
    double rtol = o->rtol, atol = o->atol;
    int max_steps = o->max_steps, k = n_steps;
    void *args[] = {&n, &ld, &dt, &k, &rtol, &atol, &max_steps, (void *)&params, &conc, (void *)&m2c,
                    &h_state, &flux, &step_flux, &counts, &step_counts, &status, &nsteps, &step_nsteps};
    const unsigned th = spec_threads(n), blocks = (unsigned)((n + th - 1) / th);
    return vk::hip_check(hipModuleLaunchKernel(t->spec_multi, blocks, 1, 1, th, 1, 1, 0, (hipStream_t)stream, args,
                                               nullptr),
                         "hipModuleLaunchKernel(vk_dopri5_spec_multi)");
}

extern "C" int vk_step_dopri5(const vk_table *t, int64_t n, int64_t ld, double dt, const vk_ode_opts *o,
                              const double *params, double *conc, const double *m2c, double *delta, double *h_state,
                              double *flux, int64_t *counts, int32_t *status, int32_t *nsteps,
                              vk_stream_t stream) {
    int rc = check_agents("vk_step_dopri5", t, n, ld);
    if (rc || n == 0) return rc;
    if (!o || !params || !conc || !m2c || !flux || (!counts && t->dev.n_ext > 0)) {
        vk::set_error("vk_step_dopri5: null argument");
        return VK_ERR_ARG;
    }
    if (!(dt > 0.0) || !(o->rtol > 0.0) || !(o->atol >= 0.0) || o->max_steps <= 0) {
        vk::set_error("vk_step_dopri5: need dt > 0, rtol > 0, atol >= 0, max_steps > 0");
        return VK_ERR_ARG;
    }
    if (o->variant == 2) {  // network-specialised kernel (vk_table_specialize)
        if (!t->spec_dopri5) {
            vk::set_error("vk_step_dopri5: variant 2 needs vk_table_specialize first");
            return VK_ERR_ARG;
        }
        double rtol = o->rtol, atol = o->atol;
        int max_steps = o->max_steps;
        void *args[] = {&n, &ld, &dt, &rtol, &atol, &max_steps, (void *)&params, &conc, (void *)&m2c,
                        &delta, &h_state, &flux, &counts, &status, &nsteps};
        const unsigned th = spec_threads(n), blocks = (unsigned)((n + th - 1) / th);
        return vk::hip_check(hipModuleLaunchKernel(t->spec_dopri5, blocks, 1, 1, th, 1, 1, 0, (hipStream_t)stream,
                                                   args, nullptr),
                             "hipModuleLaunchKernel(vk_dopri5_spec)");
    }
    if (o->variant == 3) {  // network-specialised agent per wavefront (vk_table_specialize)
        if (!t->spec_wave) {
            vk::set_error("vk_step_dopri5: variant 3 needs vk_table_specialize with a wavefront source first");
            return VK_ERR_ARG;
        }
        if (n > 0x1fffffff) {
            vk::set_error("vk_step_dopri5: agent-per-wavefront grid limited to 2^29 agents");
            return VK_ERR_LIMIT;
        }
        double rtol = o->rtol, atol = o->atol;
        int max_steps = o->max_steps;
        void *args[] = {&n, &ld, &dt, &rtol, &atol, &max_steps, (void *)&params, &conc, (void *)&m2c,
                        &delta, &h_state, &flux, &counts, &status, &nsteps};
        const int wg = t->spec_wave_waves;
        const unsigned blocks = (unsigned)((n + wg - 1) / wg);
        return vk::hip_check(hipModuleLaunchKernel(t->spec_wave, blocks, 1, 1, DW * wg, 1, 1, 0,
                                                   (hipStream_t)stream, args, nullptr),
                             "hipModuleLaunchKernel(vk_dopri5_wspec)");
    }
    const int ny = t->dev.n_dyn + t->dev.n_reactions;
    hipStream_t s = (hipStream_t)stream;
    if (o->variant == 1) {  // agent per wavefront
#define VK_DW(NS) return launch_dopri5_wave<NS>(t, n, ld, dt, o, params, conc, m2c, delta, h_state, flux, counts, status, nsteps, s)
        if (ny <= 64) VK_DW(1);
        if (ny <= 128) VK_DW(2);
        if (ny <= 256) VK_DW(4);
        if (ny <= 512) VK_DW(8);
#undef VK_DW
        vk::set_error("vk_step_dopri5: %d integrated components > 512 (agent-per-wavefront limit)", ny);
        return VK_ERR_LIMIT;
    }
    if (o->variant != 0) {
        vk::set_error("vk_step_dopri5: variant %d not available", o->variant);
        return VK_ERR_ARG;
    }
#define VK_DP(NYC) return launch_dopri5<NYC>(t, n, ld, dt, o, params, conc, m2c, delta, h_state, flux, counts, status, nsteps, s)
    switch (ny) {
        case 1: VK_DP(1); case 2: VK_DP(2); case 3: VK_DP(3); case 4: VK_DP(4);
        case 5: VK_DP(5); case 6: VK_DP(6); case 7: VK_DP(7); case 8: VK_DP(8);
        case 9: VK_DP(9); case 10: VK_DP(10); case 11: VK_DP(11); case 12: VK_DP(12);
        default: break;
    }
    if (ny <= 16) VK_DP(16);
    if (ny <= 24) VK_DP(24);
    if (ny <= 32) VK_DP(32);
#undef VK_DP
    vk::set_error("vk_step_dopri5: %d integrated components > 32 (agent-per-thread limit)", ny);
    return VK_ERR_LIMIT;
}
