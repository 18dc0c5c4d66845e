"""Test helper: evaluate a compiled RateLawTable on the CPU, one agent at a time,
in the exact operation order the HIP Euler kernel uses.

Used to check the *compiler* (host logic) against the oracle and the golden
fluxes without a GPU.  Not product code.
"""

import numpy as np


def table_fluxes(t, conc, params):
    """conc: [n_species] float64, params: [n_params] float64 -> [n_reactions]."""
    flux = [0.0] * t.n_reactions
    for l in range(t.n_rate_laws):
        num = 0.0
        for s in range(t.rl_num_ptr[l], t.rl_num_ptr[l + 1]):
            term = 1.0
            for m in range(t.set_ptr[s], t.set_ptr[s + 1]):
                km = params[t.mem_param[m]]
                term = term * (conc[t.mem_species[m]] / km if km != 0 else 0.0)
            num = num + params[t.rl_kcat[l]] * term
        num = num * conc[t.rl_enzyme[l]]
        den = 1.0
        for s in range(t.rl_den_ptr[l], t.rl_den_ptr[l + 1]):
            term = 1.0
            for m in range(t.set_ptr[s], t.set_ptr[s + 1]):
                km = params[t.mem_param[m]]
                term = term * (1.0 + conc[t.mem_species[m]] / km if km != 0 else 1.0)
            den = den + (term - 1.0)
        r = t.rl_reaction[l]
        flux[r] = flux[r] + num / den
    return np.array(flux, dtype=np.float64)


def table_euler(t, conc, params, dt, m2c):
    """One reference Euler step: returns (new conc, fluxes, counts[n_ext])."""
    flux = table_fluxes(t, conc, params)
    new = np.array(conc, dtype=np.float64)
    for s in range(t.n_dyn):
        d = 0.0
        for j in range(t.upd_ptr[s], t.upd_ptr[s + 1]):
            d = d + (t.upd_coeff[j] * flux[t.upd_rxn[j]]) * dt
        new[s] = new[s] + d
    counts = np.zeros(t.n_ext, dtype=np.int64)
    for e in range(t.n_ext):
        c = 0
        for j in range(t.ex_ptr[e], t.ex_ptr[e + 1]):
            c += int(((t.ex_coeff[j] * flux[t.ex_rxn[j]]) * dt) * m2c)
        counts[e] = c
    return new, flux, counts
