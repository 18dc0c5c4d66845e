"""Oracle for the reference's only odeint path -- TEST INFRASTRUCTURE ONLY.

Restates ``Transport.next_update`` of vivarium/processes/Kremling2007_transport.py
(the Kremling, Bettenbrock & Gilles 2007 sugar-transport model):

* the 15-component state in the reference's key order (:361-381): mass, UHPT,
  LACZ, PTSG, G6P, PEP, PYR, XP, GLC[e], G6P[e], LCTS[e] and four flux
  integrals GLCpts, PPS, PYK, glc__D_e;
* the right-hand side ``model(state, t)`` (:220-351), time in HOURS, with the
  regime switch on the *internal* G6P (``G6P > 0.01``, :245-251);
* ``odeint`` on the reference's grid ``np.arange(0, dt/3600, 0.01/3600)`` --
  100 points for dt = 1 s, the last at 0.99 s (:354-357, :384);
* outputs (:386-427): internal species := last grid row; fluxes := mean of
  the integrals over the grid rows; external changes -> counts via
  ``millimolar_to_counts`` = ``int(N_A * volume_L * (delta_mM * 1e-3))``
  (vivarium/library/flux_conversion.py:28-38), volume = global volume fL * 1e-15.

``DEFAULT_PARAMETERS`` (:19-70) and the GLC_G6P initial state (:121-133 with
vivarium/data/flat/media/GLC_G6P.tsv) are restated as data.
"""

from __future__ import annotations

import numpy as np

N_A = 6.022140857e23

DEFAULT_PARAMETERS = {
    'k1': 0.00001, 'k2': 0.0001, 'k3': 0.00016, 'K1': 3000, 'K2': 2800, 'K3': 15000,
    'kd': 0.4, 'm': 1, 'n': 2, 'x0': 0.1, 'kg6p': 2.8e6, 'Kg6p': 0.1, 'kptsup': 2.7e8,
    'Kglc': 0.12, 'Keiiap': 12, 'klac': 5.4e5, 'Km_lac': 0.13, 'Kieiia': 5.0,
    'kgly': 2.80e4, 'kpyk': 9.39e5, 'kpdh': 5.50e3, 'kpts': 1.86e5, 'km_pts': 0.7 * 1.86e5,
    'Y': 1.0e-4, 'mw1': 2.602e-4, 'mw2': 1.802e-4, 'mw3': 3.423e-4, 'Y1_sim': 6.2448e-05,
    'Y2_sim': 1.0e-4, 'Y3_sim': 9.2421e-05, 'Y4_sim': 1.0e-04, 'K': 0.4, 'kb': 600,
    'ksyn': 3.2623e3, 'KI': 1 / 8000,
}

STATE_KEYS = ('mass', 'UHPT', 'LACZ', 'PTSG', 'G6P', 'PEP', 'PYR', 'XP', 'GLC[e]', 'G6P[e]', 'LCTS[e]',
              'GLCpts', 'PPS', 'PYK', 'glc__D_e')
INTERNAL = STATE_KEYS[:8]
EXTERNAL = ('GLC[e]', 'G6P[e]', 'LCTS[e]')
FLUXES = ('GLCpts', 'PPS', 'PYK', 'glc__D_e')

# GLC_G6P condition (Kremling2007_transport.py:121-133; GLC_G6P.tsv)
GLC_G6P_INTERNAL = {'mass': 0.032, 'LACZ': 0.0, 'UHPT': 0.0003, 'PTSG': 0.007, 'G6P': 0.2057,
                    'PEP': 2.0949, 'PYR': 2.0949, 'XP': 0.0038}
GLC_G6P_EXTERNAL = {'GLC': 12.2087, 'G6P': 1.3451, 'LCTS': 0.0}
# test_transport's glucose/lactose shift condition (:433-447)
GLC_LCT_SHIFT_INTERNAL = {'mass': 0.032, 'UHPT': 1e-5, 'LACZ': 0.0, 'PTSG': 0.001, 'G6P': 0.1,
                          'PEP': 0.05, 'PYR': 0.1, 'XP': 0.01}
GLC_LCT_SHIFT_EXTERNAL = {'GLC': 0.22, 'G6P': 0.0, 'LCTS': 1.165}


def rhs(state, t, p):
    """model(state, t), Kremling2007_transport.py:220-351."""
    biomass, UHPT, LACZ, PTSG, G6P, PEP, PYR, XP, GLC_e, G6P_e, LCTS_e = state[:11]
    g6p_present = G6P > 0.01
    if g6p_present:
        sugar1, transporter1 = G6P_e, UHPT
        uptake1 = p['kg6p'] * (transporter1 * sugar1) / (p['Kg6p'] + sugar1)
    else:
        sugar1, transporter1 = LCTS_e, LACZ
        uptake1 = p['klac'] * (transporter1 * sugar1) / (
            p['Km_lac'] + sugar1 * (1 + ((p['x0'] - XP) / p['x0']) / p['Kieiia']))
    uptake2 = p['kptsup'] * XP * (PTSG * GLC_e) / (
        p['Kglc'] * p['Keiiap'] * p['x0'] + GLC_e * p['Keiiap'] * p['x0'] + XP * p['Kglc'] + XP * GLC_e)
    hill = p['kb'] + p['ksyn'] * XP ** 6 / (XP ** 6 + p['K'] ** 6)
    if g6p_present:
        synthesis1 = p['k1'] * hill * uptake1 / (p['K1'] + uptake1)
        synthesis2 = p['k2'] * (p['KI'] / (transporter1 + p['KI'])) * hill * uptake2 / (p['K2'] + uptake2)
    else:
        synthesis1 = p['k3'] * hill * uptake1 / (p['K3'] + uptake1)
        synthesis2 = p['k2'] * hill * uptake2 / (p['K2'] + uptake2)
    rgly = p['kgly'] * G6P
    rpdh = p['kpdh'] * PYR
    rpts = p['kpts'] * PEP * (p['x0'] - XP) - p['km_pts'] * PYR * XP
    f = (G6P ** p['n']) * PEP ** p['m']
    rpyk = p['kpyk'] * PEP * f
    mu = (p['Y1_sim'] if g6p_present else p['Y3_sim']) * uptake1 + p['Y2_sim'] * uptake2
    d = np.zeros(15)
    d[0] = mu * biomass
    if g6p_present:
        d[9] = -p['mw1'] * uptake1 * biomass
        d[1] = synthesis1 - (p['kd'] + mu) * transporter1
    else:
        d[10] = -p['mw3'] * uptake1 * biomass
        d[2] = synthesis1 - (p['kd'] + mu) * transporter1
    d[8] = -p['mw2'] * uptake2 * biomass
    d[3] = synthesis2 - (p['kd'] + mu) * PTSG
    d[4] = uptake1 + uptake2 - rgly
    d[5] = 2 * rgly - rpyk - rpts
    d[6] = rpyk + rpts - rpdh
    d[7] = rpts - uptake2
    d[11] = uptake2
    d[12] = uptake2
    d[13] = rpyk
    d[14] = d[9]
    return d


def initial_state(internal=GLC_G6P_INTERNAL, external=GLC_G6P_EXTERNAL):
    s = [internal[k] for k in INTERNAL] + [external['GLC'], external['G6P'], external['LCTS']] + [0.0] * 4
    return np.asarray(s, dtype=np.float64)


def grid(timestep=1.0, dt=0.01):
    return np.arange(0, timestep / 3600, dt / 3600)


def step(state0, volume_fL=1.0, timestep=1.0, params=DEFAULT_PARAMETERS, rtol=None, atol=None,
         avogadro=N_A):
    """One Transport.next_update: returns (internal[8] at the last grid row,
    mean fluxes[4] over the grid, exchange counts[3] GLC, G6P, LCTS)."""
    from scipy.integrate import odeint
    t = grid(timestep)
    kw = {}
    if rtol is not None:
        kw['rtol'] = rtol
    if atol is not None:
        kw['atol'] = atol
    sol = odeint(rhs, np.asarray(state0, dtype=np.float64), t, args=(params,), mxstep=500000, **kw)
    volume = volume_fL * 1e-15
    counts = [int(avogadro * volume * ((sol[-1, i] - sol[0, i]) * 1e-3)) for i in (8, 9, 10)]
    fluxes = [np.mean(sol[:, i]) for i in (11, 12, 13, 14)]
    return sol[-1, :8].copy(), np.array(fluxes), np.array(counts, dtype=np.int64), sol
