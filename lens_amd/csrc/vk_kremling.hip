// Kremling 2007 sugar-transport ODE, one agent per lane, adaptive DP5(4).
//
// Replaces the reference's only odeint call site: Transport.next_update,
// vivarium/processes/Kremling2007_transport.py:218-427 (RHS :220-351, grid
// :354-357, odeint :384, outputs :386-427).  The model is stiff (SURVEY §0
// finding 4): explicit DP45 needs ~290 steps per simulated second at rtol
// 1e-8, which one lane per agent absorbs with no memory traffic at all (the
// 15-component state, the 7 stages and the parameters live in registers;
// the parameters are kernel arguments -> SGPRs).
//
// Output semantics follow the reference exactly: integrate over the grid
// t_i = i * grid_h (hours), i = 0..n_grid-1 (the last point is 0.99 s for a
// 1-s step), landing on every grid point; internal species := y(t_last);
// fluxes := mean of the four flux integrals over the grid points; exchange
// counts := int(N_A * V * ((c(t_last) - c(0)) * 1e-3)) for GLC, G6P, LCTS.

#include <math.h>
#include <stdint.h>
#include <stddef.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <utility>
#include <vector>

#include "vk_internal.h"

namespace {

constexpr int KNY = 15;   // reference state: 11 species + 4 flux integrals
constexpr int KS = 11;    // species: they feed the RHS
// The four flux integrals (GLCpts, PPS, PYK, glc__D_e) never feed the RHS.
// GLCpts and PPS integrate the same rate (uptake2) from 0, so they are equal
// bit for bit and one of them is integrated (A0, counted twice in the error
// norm and written to both rows).  Their stage inputs are never read, so
// instead of seven stage vectors each keeps its 5th-order and error sums,
// accumulated as the stages complete -- the same fma chain, in the same
// order, as the species' b/e combinations.
constexpr int KA = 3;     // integrated flux integrals: A0 = GLCpts (= PPS), A1 = PYK, A2 = glc__D_e

struct Kp {  // device copy of vk_kremling_params plus host-derived constants
    double k1, k2, k3, K1, K2, K3, kd, m, n, x0, kg6p, Kg6p, kptsup, Kglc, Keiiap, klac, Km_lac, Kieiia;
    double kgly, kpyk, kpdh, kpts, km_pts, mw1, mw2, mw3, Y1_sim, Y2_sim, Y3_sim, K, kb, ksyn, KI;
    double K6;        // K**6 (host pow)
    double KglcKx0;   // Kglc * Keiiap * x0 (left to right, as the reference evaluates it)
    int n_int, m_int; // the exponents n, m when they are small non-negative integers, else -1
};

// division with the hardware reciprocal refined by one Newton step (~1e-15
// relative; tolerance parity against odeint, like every adaptive kernel here: a
// second step cost 6 % of the Kremling step, profiles/r06/r06t/)
__device__ __forceinline__ double kdiv(double a, double b) {
    double r = __builtin_amdgcn_rcp(b);
    r = fma(fma(-b, r, 1.0), r, r);
    return a * r;
}

// x**e for the model's exponents: repeated products for a small integer e
// (the reference's defaults n = 2, m = 1), pow otherwise.  EI >= 0: the exponent
// known at compile time (the kernel instantiated for it), so the products are
// straight-line code inside the RHS instead of a loop per call -- the same
// products in the same order, so the same bits.
template <int EI>
__device__ __forceinline__ double kpow(double x, double e, int ei) {
    if constexpr (EI >= 0) {
        (void)e;
        (void)ei;
        double r = 1.0;
#pragma unroll
        for (int i = 0; i < EI; ++i) r *= x;
        return r;
    } else {
        if (ei >= 0) {
            double r = 1.0;
            for (int i = 0; i < ei; ++i) r *= x;
            return r;
        }
        return pow(x, e);
    }
}

// model(state, t) in the reference's operation order (Kremling2007_transport.py:220-351)
template <int NI, int MI>
__device__ __forceinline__ void kremling_rhs(const Kp &p, const double (&s)[KS], double (&d)[KS], double (&da)[KA]) {
    const double biomass = s[0], UHPT = s[1], LACZ = s[2], PTSG = s[3], G6P = s[4], PEP = s[5], PYR = s[6],
                 XP = s[7], GLC_e = s[8], G6P_e = s[9], LCTS_e = s[10];
    const bool g6p = G6P > 0.01;
    double uptake1, transporter1;
    if (g6p) {
        transporter1 = UHPT;
        uptake1 = kdiv(p.kg6p * (transporter1 * G6P_e), p.Kg6p + G6P_e);
    } else {
        transporter1 = LACZ;
        uptake1 = kdiv(p.klac * (transporter1 * LCTS_e),
                       p.Km_lac + LCTS_e * (1.0 + kdiv(kdiv(p.x0 - XP, p.x0), p.Kieiia)));
    }
    const double uptake2 = kdiv(p.kptsup * XP * (PTSG * GLC_e),
                                p.KglcKx0 + GLC_e * p.Keiiap * p.x0 + XP * p.Kglc + XP * GLC_e);
    const double xp2 = XP * XP;
    const double xp6 = xp2 * xp2 * xp2;
    const double hill = p.kb + kdiv(p.ksyn * xp6, xp6 + p.K6);
    double synthesis1, synthesis2;
    if (g6p) {
        synthesis1 = kdiv(p.k1 * hill * uptake1, p.K1 + uptake1);
        synthesis2 = kdiv(p.k2 * kdiv(p.KI, transporter1 + p.KI) * hill * uptake2, p.K2 + uptake2);
    } else {
        synthesis1 = kdiv(p.k3 * hill * uptake1, p.K3 + uptake1);
        synthesis2 = kdiv(p.k2 * hill * uptake2, p.K2 + uptake2);
    }
    const double rgly = p.kgly * G6P;
    const double rpdh = p.kpdh * PYR;
    const double rpts = p.kpts * PEP * (p.x0 - XP) - p.km_pts * PYR * XP;
    const double f = kpow<NI>(G6P, p.n, p.n_int) * kpow<MI>(PEP, p.m, p.m_int);
    const double rpyk = p.kpyk * PEP * f;
    const double mu = (g6p ? p.Y1_sim : p.Y3_sim) * uptake1 + p.Y2_sim * uptake2;
    d[0] = mu * biomass;
    d[1] = g6p ? synthesis1 - (p.kd + mu) * transporter1 : 0.0;
    d[2] = g6p ? 0.0 : synthesis1 - (p.kd + mu) * transporter1;
    d[3] = synthesis2 - (p.kd + mu) * PTSG;
    d[4] = uptake1 + uptake2 - rgly;
    d[5] = 2.0 * rgly - rpyk - rpts;
    d[6] = rpyk + rpts - rpdh;
    d[7] = rpts - uptake2;
    d[8] = -p.mw2 * uptake2 * biomass;
    d[9] = g6p ? -p.mw1 * uptake1 * biomass : 0.0;
    d[10] = g6p ? 0.0 : -p.mw3 * uptake1 * biomass;
    da[0] = uptake2;   // GLCpts (and PPS)
    da[1] = rpyk;      // PYK
    da[2] = d[9];      // glc__D_e
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
__device__ __forceinline__ double step_factor(double en) {
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

namespace dpk {
constexpr double a21 = 1.0 / 5.0;
constexpr double a31 = 3.0 / 40.0, a32 = 9.0 / 40.0;
constexpr double a41 = 44.0 / 45.0, a42 = -56.0 / 15.0, a43 = 32.0 / 9.0;
constexpr double a51 = 19372.0 / 6561.0, a52 = -25360.0 / 2187.0, a53 = 64448.0 / 6561.0, a54 = -212.0 / 729.0;
constexpr double a61 = 9017.0 / 3168.0, a62 = -355.0 / 33.0, a63 = 46732.0 / 5247.0, a64 = 49.0 / 176.0,
                 a65 = -5103.0 / 18656.0;
constexpr double b1 = 35.0 / 384.0, b3 = 500.0 / 1113.0, b4 = 125.0 / 192.0, b5 = -2187.0 / 6784.0,
                 b6 = 11.0 / 84.0;
constexpr double e1 = 71.0 / 57600.0, e3 = -71.0 / 16695.0, e4 = 71.0 / 1920.0, e5 = -17253.0 / 339200.0,
                 e6 = 22.0 / 525.0, e7 = -1.0 / 40.0;
}  // namespace dpk

// reference component i (0..14) of the error norm: species, then A0, A0 (PPS), A1, A2
__device__ __forceinline__ int acc_of(int i) { return i == 11 || i == 12 ? 0 : i - 12; }

}  // namespace

// 2 waves per SIMD (256 VGPRs).  The parameters come through a pointer to a
// device copy, not by value: as a by-value argument they are pinned in SGPRs
// and ~1,400 SGPR spills to VGPR lanes follow; through the pointer the
// compiler re-loads them (s_load) where registers run short.
// NI / MI: the exponents n / m when the launch knows them as small integers (the
// reference's n = 2, m = 1 have an instantiation of their own), -1 otherwise.
template <int NI, int MI>
__global__ __launch_bounds__(128) __attribute__((amdgpu_waves_per_eu(2))) void k_kremling_dopri5(
                                                         const Kp *__restrict__ pp, int64_t n, int64_t ld, double grid_h, int n_grid,
                                                         double rtol, double atol, int max_steps,
                                                         double *__restrict__ state,
                                                         const double *__restrict__ volume_fl, double avogadro,
                                                         double *__restrict__ h_state, double *__restrict__ flux,
                                                         int64_t *__restrict__ counts, int32_t *__restrict__ status,
                                                         int32_t *__restrict__ nsteps_out) {
    const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= n) return;
    const Kp &p = *pp;
    double y[KS], k1[KS], k2[KS], k3[KS], k4[KS], k5[KS], k6[KS], k7[KS], yt[KS];
    double ya[KA], k1a[KA], ka[KA], s5[KA], se[KA], yta[KA];
#pragma unroll
    for (int i = 0; i < KS; ++i) y[i] = state[(int64_t)i * ld + a];
#pragma unroll
    for (int j = 0; j < KA; ++j) ya[j] = 0.0;
    const double c0_glc = y[8], c0_g6p = y[9], c0_lcts = y[10];
    kremling_rhs<NI, MI>(p, y, k1, k1a);
    int32_t st = 0;
    double h = h_state ? h_state[a] : 0.0;
    if (!(h > 0.0)) {   // scipy select_initial_step (order 4) over the first grid interval
        double d0 = 0.0, d1 = 0.0;
#pragma unroll
        for (int i = 0; i < KNY; ++i) {
            const double yi = i < KS ? y[i] : ya[acc_of(i)], fi = i < KS ? k1[i] : k1a[acc_of(i)];
            const double sc = fma(fabs(yi), rtol, atol);
            d0 = fma(yi / sc, yi / sc, d0);
            d1 = fma(fi / sc, fi / sc, d1);
        }
        d0 = sqrt(d0 / KNY);
        d1 = sqrt(d1 / KNY);
        double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 * grid_h : 0.01 * d0 / d1;
        h0 = fmin(h0, grid_h);
#pragma unroll
        for (int i = 0; i < KS; ++i) yt[i] = fma(h0, k1[i], y[i]);
        kremling_rhs<NI, MI>(p, yt, k2, ka);
        double d2 = 0.0;
#pragma unroll
        for (int i = 0; i < KNY; ++i) {
            const double yi = i < KS ? y[i] : ya[acc_of(i)];
            const double df = i < KS ? k2[i] - k1[i] : ka[acc_of(i)] - k1a[acc_of(i)];
            const double q = df / fma(fabs(yi), rtol, atol);
            d2 = fma(q, q, d2);
        }
        d2 = sqrt(d2 / KNY) / h0;
        const double h1 = (d1 <= 1e-15 && d2 <= 1e-15) ? fmax(1e-6 * grid_h, h0 * 1e-3)
                                                        : pow(0.01 / fmax(d1, d2), 0.2);
        h = fmin(100.0 * h0, h1);
    }
    double acc[4] = {0.0, 0.0, 0.0, 0.0};   // sum over grid points of the flux integrals (t_0 term is 0)
    int ns = 0;
    bool rejected = false;
    double tt = 0.0;
    for (int g = 1; g < n_grid && !st; ++g) {
        const double t_end = g * grid_h;      // np.arange: start + i * step
        while (tt < t_end) {
            if (ns >= max_steps) { st |= VK_AGENT_MAX_STEPS; break; }
            if (h < 1e-14 * grid_h) { st |= VK_AGENT_H_UNDERFLOW; break; }
            double hs = h;
            bool last = false;
            if (tt + hs >= t_end) { hs = t_end - tt; last = true; }
            ++ns;
#pragma unroll
            for (int j = 0; j < KA; ++j) { s5[j] = dpk::b1 * k1a[j]; se[j] = dpk::e1 * k1a[j]; }
#pragma unroll
            for (int i = 0; i < KS; ++i) yt[i] = fma(hs, dpk::a21 * k1[i], y[i]);
            kremling_rhs<NI, MI>(p, yt, k2, ka);                      // b2 = e2 = 0
#pragma unroll
            for (int i = 0; i < KS; ++i) yt[i] = fma(hs, fma(dpk::a32, k2[i], dpk::a31 * k1[i]), y[i]);
            kremling_rhs<NI, MI>(p, yt, k3, ka);
#pragma unroll
            for (int j = 0; j < KA; ++j) { s5[j] = fma(dpk::b3, ka[j], s5[j]); se[j] = fma(dpk::e3, ka[j], se[j]); }
#pragma unroll
            for (int i = 0; i < KS; ++i)
                yt[i] = fma(hs, fma(dpk::a43, k3[i], fma(dpk::a42, k2[i], dpk::a41 * k1[i])), y[i]);
            kremling_rhs<NI, MI>(p, yt, k4, ka);
#pragma unroll
            for (int j = 0; j < KA; ++j) { s5[j] = fma(dpk::b4, ka[j], s5[j]); se[j] = fma(dpk::e4, ka[j], se[j]); }
#pragma unroll
            for (int i = 0; i < KS; ++i)
                yt[i] = fma(hs, fma(dpk::a54, k4[i], fma(dpk::a53, k3[i], fma(dpk::a52, k2[i], dpk::a51 * k1[i]))), y[i]);
            kremling_rhs<NI, MI>(p, yt, k5, ka);
#pragma unroll
            for (int j = 0; j < KA; ++j) { s5[j] = fma(dpk::b5, ka[j], s5[j]); se[j] = fma(dpk::e5, ka[j], se[j]); }
#pragma unroll
            for (int i = 0; i < KS; ++i)
                yt[i] = fma(hs, fma(dpk::a65, k5[i], fma(dpk::a64, k4[i], fma(dpk::a63, k3[i],
                            fma(dpk::a62, k2[i], dpk::a61 * k1[i])))), y[i]);
            kremling_rhs<NI, MI>(p, yt, k6, ka);
#pragma unroll
            for (int j = 0; j < KA; ++j) {
                s5[j] = fma(dpk::b6, ka[j], s5[j]);
                se[j] = fma(dpk::e6, ka[j], se[j]);
                yta[j] = fma(hs, s5[j], ya[j]);
            }
#pragma unroll
            for (int i = 0; i < KS; ++i)
                yt[i] = fma(hs, fma(dpk::b6, k6[i], fma(dpk::b5, k5[i], fma(dpk::b4, k4[i],
                            fma(dpk::b3, k3[i], dpk::b1 * k1[i])))), y[i]);
            kremling_rhs<NI, MI>(p, yt, k7, ka);                      // FSAL: k7 is the next step's k1
#pragma unroll
            for (int j = 0; j < KA; ++j) se[j] = fma(dpk::e7, ka[j], se[j]);
            double en = 0.0;
#pragma unroll
            for (int i = 0; i < KNY; ++i) {
                double err, yo, yn;
                if (i < KS) {
                    err = hs * fma(dpk::e7, k7[i], fma(dpk::e6, k6[i], fma(dpk::e5, k5[i],
                                   fma(dpk::e4, k4[i], fma(dpk::e3, k3[i], dpk::e1 * k1[i])))));
                    yo = y[i];
                    yn = yt[i];
                } else {
                    err = hs * se[acc_of(i)];
                    yo = ya[acc_of(i)];
                    yn = yta[acc_of(i)];
                }
                const double q = kdiv(err, fma(fmax(fabs(yo), fabs(yn)), rtol, atol));
                en = fma(q, q, en);
            }
            en = sqrt(en / KNY);
            if (!isfinite(en)) { st |= VK_AGENT_NONFINITE; break; }
            if (en < 1.0) {
                double factor = (en == 0.0) ? 10.0 : fmin(10.0, 0.9 * step_factor(en));
                if (rejected) factor = fmin(1.0, factor);
                tt = last ? t_end : tt + hs;
#pragma unroll
                for (int i = 0; i < KS; ++i) { y[i] = yt[i]; k1[i] = k7[i]; }
#pragma unroll
                for (int j = 0; j < KA; ++j) { ya[j] = yta[j]; k1a[j] = ka[j]; }
                // landing on a grid point with a clipped step must not shrink h
                h = last ? fmax(h, hs * factor) : hs * factor;
                rejected = false;
            } else {
                h = hs * fmax(0.2, 0.9 * step_factor(en));
                rejected = true;
            }
        }
        acc[0] += ya[0];
        acc[1] += ya[0];
        acc[2] += ya[1];
        acc[3] += ya[2];
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
        if (!isfinite(y[i])) st |= VK_AGENT_NONFINITE;
        state[(int64_t)i * ld + a] = y[i];
    }
#pragma unroll
    for (int j = 0; j < 4; ++j) flux[(int64_t)j * ld + a] = acc[j] / n_grid;
    const double vol = volume_fl[a] * 1e-15;
    const double dc[3] = {y[8] - c0_glc, y[9] - c0_g6p, y[10] - c0_lcts};
#pragma unroll
    for (int e = 0; e < 3; ++e) {
        const double x = avogadro * vol * (dc[e] * 1e-3);
        if (!(fabs(x) < 9.2e18)) {
            st |= VK_AGENT_NONFINITE;
            counts[(int64_t)e * ld + a] = 0;
        } else {
            counts[(int64_t)e * ld + a] = (int64_t)x;
        }
    }
    if (h_state) h_state[a] = h;
    if (status) status[a] = st;
    if (nsteps_out) nsteps_out[a] = ns;
}

static int small_int(double e) {   // e as an exponent of repeated products, or -1
    return (e >= 0.0 && e <= 8.0 && e == (double)(int)e) ? (int)e : -1;
}

// Device copies of the parameter sets in use, one per (device, set), created
// at a set's first launch on that device with a synchronous copy and kept:
// colonies use a handful of sets.  The copy lives on the launch stream's
// device (hipStreamGetDevice), so two colonies on two GPUs with the same
// parameters get one copy each.  A launch being captured into a graph must
// find its set already cached (capture forbids the synchronous copy: run one
// eager step first); captured sets are pinned, since a graph keeps their
// pointers.  A parameter scan that passes more than KP_SETS_MAX distinct sets
// drains the device and frees the unpinned copies (no launch in flight can
// still read a freed copy).
constexpr size_t KP_SETS_MAX = 4096;
struct KpEntry {
    Kp p;
    int device;
    Kp *d;
    bool pinned;   // referenced by a captured graph
};
static std::mutex g_kp_mutex;
static std::vector<KpEntry> g_kp_sets;

static int device_params(const Kp &p, hipStream_t stream, const Kp **out) {
    int dev = 0;
    int rc = stream ? vk::hip_check(hipStreamGetDevice(stream, &dev), "hipStreamGetDevice")
                    : vk::hip_check(hipGetDevice(&dev), "hipGetDevice");
    if (rc) return rc;
    hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
    rc = vk::hip_check(hipStreamIsCapturing(stream, &cap), "hipStreamIsCapturing");
    if (rc) return rc;
    const bool capturing = cap != hipStreamCaptureStatusNone;
    std::lock_guard<std::mutex> lock(g_kp_mutex);
    for (auto &e : g_kp_sets)
        if (e.device == dev && memcmp(&e.p, &p, sizeof(Kp)) == 0) {
            e.pinned |= capturing;
            *out = e.d;
            return VK_OK;
        }
    if (capturing) {
        vk::set_error("vk_kremling_step: a parameter set seen for the first time during graph capture "
                      "(its device copy is synchronous); run one eager step with it before capturing");
        return VK_ERR_ARG;
    }
    int prev = 0;
    rc = vk::hip_check(hipGetDevice(&prev), "hipGetDevice");
    if (rc) return rc;
    if (prev != dev && (rc = vk::hip_check(hipSetDevice(dev), "hipSetDevice"))) return rc;
    if (g_kp_sets.size() >= KP_SETS_MAX) {
        for (auto &e : g_kp_sets) {
            if (e.pinned) continue;
            if ((rc = vk::hip_check(hipSetDevice(e.device), "hipSetDevice")) ||
                (rc = vk::hip_check(hipDeviceSynchronize(), "hipDeviceSynchronize(kremling params)")))
                break;
            (void)hipFree(e.d);
            e.d = nullptr;
        }
        g_kp_sets.erase(std::remove_if(g_kp_sets.begin(), g_kp_sets.end(),
                                       [](const KpEntry &e) { return e.d == nullptr; }),
                        g_kp_sets.end());
        if (!rc) rc = vk::hip_check(hipSetDevice(dev), "hipSetDevice");
    }
    Kp *d = nullptr;
    if (!rc) rc = vk::hip_check(hipMalloc(&d, sizeof(Kp)), "hipMalloc(kremling params)");
    if (!rc) {
        rc = vk::hip_check(hipMemcpy(d, &p, sizeof(Kp), hipMemcpyHostToDevice), "hipMemcpy(kremling params)");
        if (rc) (void)hipFree(d);
    }
    if (prev != dev) (void)hipSetDevice(prev);
    if (rc) return rc;
    g_kp_sets.push_back(KpEntry{p, dev, d, false});
    *out = d;
    return VK_OK;
}

extern "C" int vk_kremling_step(const vk_kremling_params *kp, int64_t n, int64_t ld, double timestep_h,
                                double grid_h, int32_t n_grid, double rtol, double atol, int32_t max_steps,
                                double *state, const double *volume_fl, double avogadro, double *h_state,
                                double *flux, int64_t *counts, int32_t *status, int32_t *nsteps,
                                vk_stream_t stream) {
    if (!kp || n < 0 || ld < n || n_grid < 1 || !(grid_h > 0.0) || !(rtol > 0.0) || !(atol >= 0.0) ||
        max_steps <= 0 || (n > 0 && (!state || !volume_fl || !flux || !counts))) {
        vk::set_error("vk_kremling_step: bad arguments");
        return VK_ERR_ARG;
    }
    (void)timestep_h;
    if (n == 0) return VK_OK;
    Kp p;
    memset(&p, 0, sizeof(Kp));   // padding too: parameter sets are compared bytewise
    static_assert(offsetof(Kp, K6) == sizeof(vk_kremling_params), "parameter layout");
    memcpy(&p, kp, sizeof(vk_kremling_params));
    p.K6 = pow(kp->K, 6.0);
    p.KglcKx0 = kp->Kglc * kp->Keiiap * kp->x0;
    p.n_int = small_int(kp->n);
    p.m_int = small_int(kp->m);
    const Kp *dp = nullptr;
    int rc = device_params(p, (hipStream_t)stream, &dp);
    if (rc) return rc;
    auto kern = (p.n_int == 2 && p.m_int == 1) ? k_kremling_dopri5<2, 1> : k_kremling_dopri5<-1, -1>;
    hipLaunchKernelGGL(kern, dim3((unsigned)((n + 127) / 128)), dim3(128), 0, (hipStream_t)stream, dp,
                       n, ld, grid_h, n_grid, rtol, atol, max_steps, state, volume_fl, avogadro, h_state, flux,
                       counts, status, nsteps);
    return vk::launch_check("k_kremling_dopri5");
}
