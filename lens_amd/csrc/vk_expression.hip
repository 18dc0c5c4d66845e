// ODE gene expression with boolean regulation, one agent per lane.
//
// ODE_expression.next_update (vivarium/processes/ode_expression.py:265-303):
// transcripts dM = (k_M - d_M*M)*dt unless their regulation rule holds
// (then the leak magnitude or 0), proteins dP = (k_P*m - d_P*P)*dt, all from
// the step-start state.  Rules (vivarium/library/regulation_logic.py) arrive
// as postfix programs evaluated with a bit stack; a program is the same for
// every agent, so its walk is wave-uniform (scalar-cache loads).

#include <stdint.h>

#include "vk_internal.h"

__global__ __launch_bounds__(256) void k_expression_step(vk_expr_table t, int64_t n, int64_t ld, double dt,
                                                         double *__restrict__ conc, double *__restrict__ update,
                                                         const double *__restrict__ u, int accumulate) {
    const int64_t a = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (a >= n) return;
    for (int j = 0; j < t.n_tx; ++j) {
        double rate = ldc(t.tx_rate, j);
        const int p0 = ldc(t.tx_prog_ptr, j), p1 = ldc(t.tx_prog_ptr, j + 1);
        if (p1 > p0) {
            uint32_t stack = 0;   // bit stack, top = bit 0
            for (int k = p0; k < p1; ++k) {
                const int op = ldc(t.code, 3 * k), x = ldc(t.code, 3 * k + 1), y = ldc(t.code, 3 * k + 2);
                if (op == VK_EXPR_NOT) {
                    stack ^= 1u;
                    continue;
                }
                uint32_t bit;
                if (op == VK_EXPR_CMP_GT) {
                    bit = conc[(int64_t)x * ld + a] > ldc(t.thr, y);
                } else if (op == VK_EXPR_CMP_LT) {
                    bit = conc[(int64_t)x * ld + a] < ldc(t.thr, y);
                } else if (op == VK_EXPR_PRESENT) {
                    bit = conc[(int64_t)x * ld + a] > 0.0;
                } else if (op == VK_EXPR_CONST) {
                    bit = x != 0;
                } else {   // AND / OR pop two
                    const uint32_t rhs = stack & 1u, lhs = (stack >> 1) & 1u;
                    stack >>= 2;
                    bit = (op == VK_EXPR_AND) ? (lhs & rhs) : (lhs | rhs);
                }
                stack = (stack << 1) | bit;
            }
            if (stack & 1u) {   // inhibited: leak or nothing (ode_expression.py:279-286)
                const bool leak = u && t.leak_p > 0.0 && u[(int64_t)j * ld + a] < t.leak_p;
                rate = leak ? t.leak_magnitude : 0.0;
            }
        }
        const double m = conc[(int64_t)ldc(t.tx_row, j) * ld + a];
        update[(int64_t)j * ld + a] = (rate - ldc(t.tx_deg, j) * m) * dt;
    }
    for (int j = 0; j < t.n_tl; ++j) {
        const double m = conc[(int64_t)ldc(t.tl_mrna_row, j) * ld + a];
        const double p = conc[(int64_t)ldc(t.tl_row, j) * ld + a];
        update[(int64_t)(t.n_tx + j) * ld + a] = (ldc(t.tl_rate, j) * m - ldc(t.tl_deg, j) * p) * dt;
    }
    if (accumulate) {   // the accumulate updater, after every value came from the step-start state
        for (int j = 0; j < t.n_tx; ++j) {
            const int64_t r = (int64_t)ldc(t.tx_row, j) * ld + a;
            conc[r] = conc[r] + update[(int64_t)j * ld + a];
        }
        for (int j = 0; j < t.n_tl; ++j) {
            const int64_t r = (int64_t)ldc(t.tl_row, j) * ld + a;
            conc[r] = conc[r] + update[(int64_t)(t.n_tx + j) * ld + a];
        }
    }
}

extern "C" int vk_expression_step(const vk_expr_table *t, int64_t n, int64_t ld, double dt, double *conc,
                                  double *update, const double *u, int32_t accumulate, vk_stream_t stream) {
    if (!t || n < 0 || ld < n || t->n_tx < 0 || t->n_tl < 0 ||
        (n > 0 && (!conc || !update || (t->n_tx && (!t->tx_row || !t->tx_rate || !t->tx_deg || !t->tx_prog_ptr)) ||
                   (t->n_tl && (!t->tl_row || !t->tl_mrna_row || !t->tl_rate || !t->tl_deg))))) {
        vk::set_error("vk_expression_step: bad arguments");
        return VK_ERR_ARG;
    }
    if (n == 0) return VK_OK;
    hipLaunchKernelGGL(k_expression_step, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, (hipStream_t)stream, *t, n,
                       ld, dt, conc, update, u, accumulate);
    return vk::launch_check("k_expression_step");
}
