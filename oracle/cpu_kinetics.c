/*
 * Oracle + CPU baseline (TEST INFRASTRUCTURE ONLY; never linked into lens_amd).
 *
 * A C restatement of the hot path, OpenMP over agents / rows:
 *   oc_rate_fluxes, oc_step_euler -- kinetic_rate_laws.py:149-178, :277-297 and
 *       convenience_kinetics.py:320-349, in the reference's operation order
 *   oc_step_dopri5 -- adaptive Dormand-Prince 5(4) with scipy RK45 step control
 *       (scipy/integrate/_ivp/rk.py semantics: select_initial_step, RMS error
 *       norm, SAFETY 0.9, factors [0.2, 10], no growth right after a reject)
 *       on the augmented system [internal species | flux integrals]
 *   oc_diffuse -- diffusion_field.py:385-394 with scipy convolve's summation
 *       order (up, left, -4*centre, right, down), reflect boundary
 *   oc_exchange -- registry.py:149-183 applied agent by agent
 * The table layout is the vk_table_desc of include/vk_kinetics.h (host arrays).
 * Built by oracle/Makefile into oracle/liblens_oracle.so.
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "vk_kinetics.h"

#define T (*t)

static double rate_law_exact(const vk_table_desc *t, int l, const double *params,
                             const double *conc, int64_t ld, int64_t a) {
    double num = 0.0;
    for (int s = T.rl_num_ptr[l]; s < T.rl_num_ptr[l + 1]; ++s) {
        double term = 1.0;
        for (int m = T.set_ptr[s]; m < T.set_ptr[s + 1]; ++m) {
            double km = params[(int64_t)T.mem_param[m] * ld + a];
            double c = conc[(int64_t)T.mem_species[m] * ld + a];
            term = term * (km != 0.0 ? c / km : 0.0);
        }
        num = num + params[(int64_t)T.rl_kcat[l] * ld + a] * term;
    }
    num = num * conc[(int64_t)T.rl_enzyme[l] * ld + a];
    double den = 1.0;
    for (int s = T.rl_den_ptr[l]; s < T.rl_den_ptr[l + 1]; ++s) {
        double term = 1.0;
        for (int m = T.set_ptr[s]; m < T.set_ptr[s + 1]; ++m) {
            double km = params[(int64_t)T.mem_param[m] * ld + a];
            double c = conc[(int64_t)T.mem_species[m] * ld + a];
            term = term * (km != 0.0 ? 1.0 + c / km : 1.0);
        }
        den = den + (term - 1.0);
    }
    return num / den;
}

void oc_rate_fluxes(const vk_table_desc *t, int64_t n, int64_t ld, const double *params,
                    const double *conc, double *flux) {
#pragma omp parallel for schedule(static)
    for (int64_t a = 0; a < n; ++a) {
        for (int r = 0; r < T.n_reactions; ++r) flux[(int64_t)r * ld + a] = 0.0;
        for (int l = 0; l < T.n_rate_laws; ++l) {
            int64_t idx = (int64_t)T.rl_reaction[l] * ld + a;
            flux[idx] = flux[idx] + rate_law_exact(t, l, params, conc, ld, a);
        }
    }
}

void oc_step_euler(const vk_table_desc *t, int64_t n, int64_t ld, double dt, const double *params,
                   double *conc, const double *m2c, double *flux, int64_t *counts) {
    oc_rate_fluxes(t, n, ld, params, conc, flux);
#pragma omp parallel for schedule(static)
    for (int64_t a = 0; a < n; ++a) {
        for (int s = 0; s < T.n_dyn; ++s) {
            double d = 0.0;
            for (int j = T.upd_ptr[s]; j < T.upd_ptr[s + 1]; ++j)
                d = d + (T.upd_coeff[j] * flux[(int64_t)T.upd_rxn[j] * ld + a]) * dt;
            conc[(int64_t)s * ld + a] = conc[(int64_t)s * ld + a] + d;
        }
        for (int e = 0; e < T.n_ext; ++e) {
            int64_t c = 0;
            for (int j = T.ex_ptr[e]; j < T.ex_ptr[e + 1]; ++j)
                c += (int64_t)(((T.ex_coeff[j] * flux[(int64_t)T.ex_rxn[j] * ld + a]) * dt) * m2c[a]);
            counts[(int64_t)e * ld + a] = c;
        }
    }
}

/* ---- DP5(4): y = [dyn | integrals], per agent, scratch on the stack ---- */

typedef struct {
    const vk_table_desc *t;
    double *c;      /* [n_species] species (dyn rows overwritten per stage) */
    double *p;      /* [n_params] kcat or 1/Km */
    double *f;      /* [n_reactions] fluxes */
} agent_ctx;

static void rhs(const agent_ctx *x, const double *y, double *dy) {
    const vk_table_desc *t = x->t;
    int nd = T.n_dyn, R = T.n_reactions;
    for (int i = 0; i < nd; ++i) x->c[i] = y[i];
    for (int r = 0; r < R; ++r) x->f[r] = 0.0;
    for (int l = 0; l < T.n_rate_laws; ++l) {
        double num = 0.0;
        for (int s = T.rl_num_ptr[l]; s < T.rl_num_ptr[l + 1]; ++s) {
            double term = x->p[T.rl_kcat[l]];
            for (int m = T.set_ptr[s]; m < T.set_ptr[s + 1]; ++m)
                term *= x->c[T.mem_species[m]] * x->p[T.mem_param[m]];
            num += term;
        }
        num *= x->c[T.rl_enzyme[l]];
        double den = 1.0;
        for (int s = T.rl_den_ptr[l]; s < T.rl_den_ptr[l + 1]; ++s) {
            double term = 1.0;
            for (int m = T.set_ptr[s]; m < T.set_ptr[s + 1]; ++m)
                term *= fma(x->c[T.mem_species[m]], x->p[T.mem_param[m]], 1.0);
            den += term - 1.0;
        }
        x->f[T.rl_reaction[l]] += num / den;
    }
    for (int i = 0; i < nd; ++i) {
        double d = 0.0;
        for (int j = T.upd_ptr[i]; j < T.upd_ptr[i + 1]; ++j) d = fma(T.upd_coeff[j], x->f[T.upd_rxn[j]], d);
        dy[i] = d;
    }
    for (int r = 0; r < R; ++r) dy[nd + r] = x->f[r];
}

static double rms(const double *v, const double *sc, int ny) {
    double s = 0.0;
    for (int i = 0; i < ny; ++i) {
        double q = v[i] / sc[i];
        s = fma(q, q, s);
    }
    return sqrt(s / ny);
}

int oc_step_dopri5(const vk_table_desc *t, int64_t n, int64_t ld, double dt, double rtol, double atol,
                   int max_steps, const double *params, double *conc, const double *m2c,
                   double *h_state, double *flux, int64_t *counts, int32_t *status, int32_t *nsteps) {
    const double a21 = 1.0 / 5.0, a31 = 3.0 / 40.0, a32 = 9.0 / 40.0, a41 = 44.0 / 45.0,
                 a42 = -56.0 / 15.0, a43 = 32.0 / 9.0, a51 = 19372.0 / 6561.0, a52 = -25360.0 / 2187.0,
                 a53 = 64448.0 / 6561.0, a54 = -212.0 / 729.0, a61 = 9017.0 / 3168.0, a62 = -355.0 / 33.0,
                 a63 = 46732.0 / 5247.0, a64 = 49.0 / 176.0, a65 = -5103.0 / 18656.0, b1 = 35.0 / 384.0,
                 b3 = 500.0 / 1113.0, b4 = 125.0 / 192.0, b5 = -2187.0 / 6784.0, b6 = 11.0 / 84.0,
                 e1 = 71.0 / 57600.0, e3 = -71.0 / 16695.0, e4 = 71.0 / 1920.0,
                 e5 = -17253.0 / 339200.0, e6 = 22.0 / 525.0, e7 = -1.0 / 40.0;
    const int nd = T.n_dyn, R = T.n_reactions, ny = nd + R, S = T.n_species, P = T.n_params;
    const int n_members = T.set_ptr[T.rl_den_ptr[T.n_rate_laws]];
    int fail = 0;
#pragma omp parallel reduction(| : fail)
    {
        double *buf = (double *)malloc(sizeof(double) * (S + P + R + 10 * ny));
        agent_ctx x = {t, buf, buf + S, buf + S + P};
        double *y = buf + S + P + R, *k1 = y + ny, *k2 = k1 + ny, *k3 = k2 + ny, *k4 = k3 + ny,
               *k5 = k4 + ny, *k6 = k5 + ny, *k7 = k6 + ny, *yt = k7 + ny, *sc = yt + ny;
#pragma omp for schedule(dynamic, 64)
        for (int64_t a = 0; a < n; ++a) {
            for (int s = 0; s < S; ++s) x.c[s] = conc[(int64_t)s * ld + a];
            for (int q = 0; q < P; ++q) x.p[q] = params[(int64_t)q * ld + a];
            for (int m = 0; m < n_members; ++m) {
                double km = params[(int64_t)T.mem_param[m] * ld + a];
                x.p[T.mem_param[m]] = km != 0.0 ? 1.0 / km : 0.0;
            }
            for (int i = 0; i < ny; ++i) y[i] = i < nd ? x.c[i] : 0.0;
            rhs(&x, y, k1);
            int32_t st = 0;
            double h = h_state ? h_state[a] : 0.0;
            if (!(h > 0.0)) {
                for (int i = 0; i < ny; ++i) sc[i] = fma(fabs(y[i]), rtol, atol);
                double d0 = rms(y, sc, ny), d1 = rms(k1, sc, ny);
                double h0 = (d0 < 1e-5 || d1 < 1e-5) ? 1e-6 : 0.01 * d0 / d1;
                h0 = fmin(h0, dt);
                for (int i = 0; i < ny; ++i) yt[i] = fma(h0, k1[i], y[i]);
                rhs(&x, yt, k2);
                for (int i = 0; i < ny; ++i) k2[i] = k2[i] - k1[i];
                double d2 = rms(k2, sc, ny) / h0;
                double h1 = (d1 <= 1e-15 && d2 <= 1e-15) ? fmax(1e-6, h0 * 1e-3) : pow(0.01 / fmax(d1, d2), 0.2);
                h = fmin(fmin(100.0 * h0, h1), dt);
            }
            double tt = 0.0, h_keep = h;
            int ns = 0, rejected = 0;
            while (tt < dt) {
                if (ns >= max_steps) { st |= VK_AGENT_MAX_STEPS; break; }
                if (h < 1e-14 * dt) { st |= VK_AGENT_H_UNDERFLOW; break; }
                double hs = h;
                int last = 0;
                if (tt + hs >= dt) { hs = dt - tt; last = 1; }
                ++ns;
                for (int i = 0; i < ny; ++i) yt[i] = fma(hs, a21 * k1[i], y[i]);
                rhs(&x, yt, k2);
                for (int i = 0; i < ny; ++i) yt[i] = fma(hs, fma(a32, k2[i], a31 * k1[i]), y[i]);
                rhs(&x, yt, k3);
                for (int i = 0; i < ny; ++i) yt[i] = fma(hs, fma(a43, k3[i], fma(a42, k2[i], a41 * k1[i])), y[i]);
                rhs(&x, yt, k4);
                for (int i = 0; i < ny; ++i)
                    yt[i] = fma(hs, fma(a54, k4[i], fma(a53, k3[i], fma(a52, k2[i], a51 * k1[i]))), y[i]);
                rhs(&x, yt, k5);
                for (int i = 0; i < ny; ++i)
                    yt[i] = fma(hs, fma(a65, k5[i], fma(a64, k4[i], fma(a63, k3[i], fma(a62, k2[i], a61 * k1[i])))), y[i]);
                rhs(&x, yt, k6);
                for (int i = 0; i < ny; ++i)
                    yt[i] = fma(hs, fma(b6, k6[i], fma(b5, k5[i], fma(b4, k4[i], fma(b3, k3[i], b1 * k1[i])))), y[i]);
                rhs(&x, yt, k7);
                double en = 0.0;
                for (int i = 0; i < ny; ++i) {
                    double err = hs * fma(e7, k7[i], fma(e6, k6[i], fma(e5, k5[i], fma(e4, k4[i], fma(e3, k3[i], e1 * k1[i])))));
                    double q = err / fma(fmax(fabs(y[i]), fabs(yt[i])), rtol, atol);
                    en = fma(q, q, en);
                }
                en = sqrt(en / ny);
                if (!isfinite(en)) { st |= VK_AGENT_NONFINITE; break; }
                if (en < 1.0) {
                    double factor = en == 0.0 ? 10.0 : fmin(10.0, 0.9 * pow(en, -0.2));
                    if (rejected) factor = fmin(1.0, factor);
                    tt = last ? dt : tt + hs;
                    memcpy(y, yt, sizeof(double) * ny);
                    memcpy(k1, k7, sizeof(double) * ny);
                    h_keep = last ? fmax(h, hs * factor) : hs * factor;
                    h = hs * factor;
                    rejected = 0;
                } else {
                    h = hs * fmax(0.2, 0.9 * pow(en, -0.2));
                    rejected = 1;
                }
            }
            for (int i = 0; i < nd; ++i) conc[(int64_t)i * ld + a] = y[i];
            for (int r = 0; r < R; ++r) flux[(int64_t)r * ld + a] = y[nd + r] / dt;
            for (int e = 0; e < T.n_ext; ++e) {
                int64_t c = 0;
                for (int j = T.ex_ptr[e]; j < T.ex_ptr[e + 1]; ++j)
                    c += (int64_t)((T.ex_coeff[j] * y[nd + T.ex_rxn[j]]) * m2c[a]);
                counts[(int64_t)e * ld + a] = c;
            }
            if (h_state) h_state[a] = h_keep;
            if (status) status[a] = st;
            if (nsteps) nsteps[a] = ns;
            if (st) fail = 1;
        }
        free(buf);
    }
    return fail;
}

/* ---- lattice ---- */

static void substep(const double *src, double *dst, const double *f0, int nx, int ny, double coef) {
#pragma omp parallel for schedule(static)
    for (int r = 0; r < nx; ++r) {
        const double *up = src + (int64_t)(r > 0 ? r - 1 : 0) * ny;
        const double *mid = src + (int64_t)r * ny;
        const double *dn = src + (int64_t)(r < nx - 1 ? r + 1 : nx - 1) * ny;
        double *out = dst + (int64_t)r * ny;
        const double *base = f0 ? f0 + (int64_t)r * ny : 0;
        for (int j = 0; j < ny; ++j) {
            double l = mid[j > 0 ? j - 1 : 0], rr = mid[j < ny - 1 ? j + 1 : ny - 1];
            double lap = (((up[j] + l) + (-4.0 * mid[j])) + rr) + dn[j];
            double v = mid[j] + coef * lap;
            if (base) v = base[j] + (v - base[j]);
            out[j] = v;
        }
    }
}

/* n_sub substeps of one plane; the last writes field = field + (new - field).
 * Uniform planes are skipped (diffusion_field.py:401-404). */
void oc_diffuse(double *field, double *w0, double *w1, int nx, int ny, double coef, int n_sub) {
    int64_t cells = (int64_t)nx * ny;
    int uniform = 1;
    for (int64_t i = 1; i < cells && uniform; ++i) uniform = field[i] == field[0];
    if (uniform || n_sub <= 0) return;
    double *w[2] = {w0, w1};
    for (int j = 0; j < n_sub; ++j) {
        const double *src = j == 0 ? field : w[(j - 1) & 1];
        if (j == n_sub - 1) {
            double *dst = (j == 0) ? w0 : field;
            substep(src, dst, field, nx, ny, coef);
            if (j == 0) memcpy(field, w0, sizeof(double) * cells);
        } else {
            substep(src, w[j & 1], 0, nx, ny, coef);
        }
    }
}

/* agent-ordered exchange into one plane (bin_lin per agent) */
void oc_exchange(double *field, const int32_t *bin_lin, const int64_t *counts, int64_t n,
                 double binvol_avogadro) {
    for (int64_t a = 0; a < n; ++a)
        field[bin_lin[a]] = field[bin_lin[a]] + ((double)counts[a] / binvol_avogadro) * 1000.0;
}
