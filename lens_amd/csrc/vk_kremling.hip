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
#include <string.h>

#include "vk_internal.h"

namespace {

constexpr int KNY = 15;

struct Kp {  // device copy of vk_kremling_params
    double k1, k2, k3, K1, K2, K3, kd, m, n, x0, kg6p, Kg6p, kptsup, Kglc, Keiiap, klac, Km_lac, Kieiia;
    double kgly, kpyk, kpdh, kpts, km_pts, mw1, mw2, mw3, Y1_sim, Y2_sim, Y3_sim, K, kb, ksyn, KI;
};

// model(state, t) in the reference's operation order
__device__ __forceinline__ void kremling_rhs(const Kp &p, const double (&s)[KNY], double (&d)[KNY]) {
    const double biomass = s[0], UHPT = s[1], LACZ = s[2], PTSG = s[3], G6P = s[4], PEP = s[5], PYR = s[6],
                 XP = s[7], GLC_e = s[8], G6P_e = s[9], LCTS_e = s[10];
    const bool g6p = G6P > 0.01;
    double uptake1, transporter1;
    if (g6p) {
        transporter1 = UHPT;
        uptake1 = p.kg6p * (transporter1 * G6P_e) / (p.Kg6p + G6P_e);
    } else {
        transporter1 = LACZ;
        uptake1 = p.klac * (transporter1 * LCTS_e) /
                  (p.Km_lac + LCTS_e * (1.0 + ((p.x0 - XP) / p.x0) / p.Kieiia));
    }
    const double uptake2 = p.kptsup * XP * (PTSG * GLC_e) /
                           (p.Kglc * p.Keiiap * p.x0 + GLC_e * p.Keiiap * p.x0 + XP * p.Kglc + XP * GLC_e);
    const double xp6 = pow(XP, 6.0);
    const double hill = p.kb + p.ksyn * xp6 / (xp6 + pow(p.K, 6.0));
    double synthesis1, synthesis2;
    if (g6p) {
        synthesis1 = p.k1 * hill * uptake1 / (p.K1 + uptake1);
        synthesis2 = p.k2 * (p.KI / (transporter1 + p.KI)) * hill * uptake2 / (p.K2 + uptake2);
    } else {
        synthesis1 = p.k3 * hill * uptake1 / (p.K3 + uptake1);
        synthesis2 = p.k2 * hill * uptake2 / (p.K2 + uptake2);
    }
    const double rgly = p.kgly * G6P;
    const double rpdh = p.kpdh * PYR;
    const double rpts = p.kpts * PEP * (p.x0 - XP) - p.km_pts * PYR * XP;
    const double f = pow(G6P, p.n) * pow(PEP, p.m);
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
    d[11] = uptake2;
    d[12] = uptake2;
    d[13] = rpyk;
    d[14] = d[9];
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

}  // namespace

__global__ __launch_bounds__(128) void k_kremling_dopri5(Kp p, int64_t n, int64_t ld, double grid_h, int n_grid,
                                                         double rtol, double atol, int max_steps,
                                                         double *__restrict__ state,
                                                         const double *__restrict__ volume_fl, double avogadro,
                                                         double *__restrict__ h_state, double *__restrict__ flux,
                                                         int64_t *__restrict__ counts, int32_t *__restrict__ status,
                                                         int32_t *__restrict__ nsteps_out) {
    const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= n) return;
    double y[KNY], k1[KNY], k2[KNY], k3[KNY], k4[KNY], k5[KNY], k6[KNY], k7[KNY], yt[KNY];
#pragma unroll
    for (int i = 0; i < 11; ++i) y[i] = state[(int64_t)i * ld + a];
#pragma unroll
    for (int i = 11; i < KNY; ++i) y[i] = 0.0;
    const double c0_glc = y[8], c0_g6p = y[9], c0_lcts = y[10];
    kremling_rhs(p, y, k1);
    int32_t st = 0;
    double h = h_state ? h_state[a] : 0.0;
    if (!(h > 0.0)) {   // scipy select_initial_step (order 4) over the first grid interval
        double d0 = 0.0, d1 = 0.0;
#pragma unroll
        for (int i = 0; i < KNY; ++i) {
            const double sc = fma(fabs(y[i]), rtol, atol);
            d0 = fma(y[i] / sc, y[i] / sc, d0);
            d1 = fma(k1[i] / sc, k1[i] / sc, d1);
        }
        d0 = sqrt(d0 / KNY);
        d1 = sqrt(d1 / KNY);
        double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 * grid_h : 0.01 * d0 / d1;
        h0 = fmin(h0, grid_h);
#pragma unroll
        for (int i = 0; i < KNY; ++i) yt[i] = fma(h0, k1[i], y[i]);
        kremling_rhs(p, yt, k2);
        double d2 = 0.0;
#pragma unroll
        for (int i = 0; i < KNY; ++i) {
            const double q = (k2[i] - k1[i]) / fma(fabs(y[i]), rtol, atol);
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
            for (int i = 0; i < KNY; ++i) yt[i] = fma(hs, dpk::a21 * k1[i], y[i]);
            kremling_rhs(p, yt, k2);
#pragma unroll
            for (int i = 0; i < KNY; ++i) yt[i] = fma(hs, fma(dpk::a32, k2[i], dpk::a31 * k1[i]), y[i]);
            kremling_rhs(p, yt, k3);
#pragma unroll
            for (int i = 0; i < KNY; ++i)
                yt[i] = fma(hs, fma(dpk::a43, k3[i], fma(dpk::a42, k2[i], dpk::a41 * k1[i])), y[i]);
            kremling_rhs(p, yt, k4);
#pragma unroll
            for (int i = 0; i < KNY; ++i)
                yt[i] = fma(hs, fma(dpk::a54, k4[i], fma(dpk::a53, k3[i], fma(dpk::a52, k2[i], dpk::a51 * k1[i]))), y[i]);
            kremling_rhs(p, yt, k5);
#pragma unroll
            for (int i = 0; i < KNY; ++i)
                yt[i] = fma(hs, fma(dpk::a65, k5[i], fma(dpk::a64, k4[i], fma(dpk::a63, k3[i],
                            fma(dpk::a62, k2[i], dpk::a61 * k1[i])))), y[i]);
            kremling_rhs(p, yt, k6);
#pragma unroll
            for (int i = 0; i < KNY; ++i)
                yt[i] = fma(hs, fma(dpk::b6, k6[i], fma(dpk::b5, k5[i], fma(dpk::b4, k4[i],
                            fma(dpk::b3, k3[i], dpk::b1 * k1[i])))), y[i]);
            kremling_rhs(p, yt, k7);
            double en = 0.0;
#pragma unroll
            for (int i = 0; i < KNY; ++i) {
                const double err = hs * fma(dpk::e7, k7[i], fma(dpk::e6, k6[i], fma(dpk::e5, k5[i],
                                       fma(dpk::e4, k4[i], fma(dpk::e3, k3[i], dpk::e1 * k1[i])))));
                const double q = err / fma(fmax(fabs(y[i]), fabs(yt[i])), rtol, atol);
                en = fma(q, q, en);
            }
            en = sqrt(en / KNY);
            if (!isfinite(en)) { st |= VK_AGENT_NONFINITE; break; }
            if (en < 1.0) {
                double factor = (en == 0.0) ? 10.0 : fmin(10.0, 0.9 * pow(en, -0.2));
                if (rejected) factor = fmin(1.0, factor);
                tt = last ? t_end : tt + hs;
#pragma unroll
                for (int i = 0; i < KNY; ++i) { y[i] = yt[i]; k1[i] = k7[i]; }
                // landing on a grid point with a clipped step must not shrink h
                h = last ? fmax(h, hs * factor) : hs * factor;
                rejected = false;
            } else {
                h = hs * fmax(0.2, 0.9 * pow(en, -0.2));
                rejected = true;
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[j] += y[11 + j];
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
    static_assert(sizeof(Kp) == sizeof(vk_kremling_params), "parameter layout");
    memcpy(&p, kp, sizeof(Kp));
    hipLaunchKernelGGL(k_kremling_dopri5, dim3((unsigned)((n + 127) / 128)), dim3(128), 0, (hipStream_t)stream, p,
                       n, ld, grid_h, n_grid, rtol, atol, max_steps, state, volume_fl, avogadro, h_state, flux,
                       counts, status, nsteps);
    return vk::launch_check("k_kremling_dopri5");
}
