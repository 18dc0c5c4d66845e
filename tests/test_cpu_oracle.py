"""The C restatement (CPU baseline) agrees with the pinned Python oracle."""

import os

import numpy as np
import pytest

from netcodec import decode_network, decode_conc
from lens_amd.rate_law_compiler import compile_rate_laws
from lens_amd import configs
from oracle import cpu
from oracle.kinetics import OracleODE, mmol_to_counts
from oracle import lattice as olat

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


def _soa(t, concs):
    return np.ascontiguousarray(np.array([[float(c.get(k, 0.0)) for c in concs] for k in t.species]))


def test_c_fluxes_bitwise(golden_fluxes):
    for case in golden_fluxes['cases']:
        rx, kp = decode_network(case['network'])
        t = compile_rate_laws(rx, kp)
        concs = [decode_conc(c) for c in case['concs']]
        conc = _soa(t, concs)
        params = np.ascontiguousarray(np.repeat(t.param_defaults[:, None], len(concs), axis=1))
        flux = cpu.rate_fluxes(cpu.Desc(t), params, conc)
        expect = np.array([[f[r] for f in case['fluxes']] for r in t.reaction_ids])
        assert np.array_equal(flux, expect), case['name']


def test_c_dopri5_matches_odeint():
    cfg = configs.glc_lct_config()
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    params, conc = configs.heterogeneous_colony(t, cfg, 64, seed=7)
    m2c = np.full(64, mmol_to_counts())
    c0 = conc.copy()
    flux, counts, status, nsteps = cpu.step_dopri5(cpu.Desc(t), 1.0, params, conc, m2c)
    assert not status.any() and nsteps.min() >= 1
    for a in range(0, 64, 9):
        rx = {r: dict(cfg['reactions'][r]) for r in cfg['reactions']}
        kp = {}
        for (kind, rid, enz, *mol), v in zip(t.param_names, params[:, a]):
            kp.setdefault(rid, {}).setdefault(enz, {})
            kp[rid][enz]['kcat_f' if kind == 'kcat' else mol[0]] = float(v)
        for rid in cfg['kinetic_parameters']:   # keep the None (non-limiting) entries
            for enz, p in cfg['kinetic_parameters'][rid].items():
                for k, v in p.items():
                    if v is None:
                        kp[rid][enz][k] = None
        ode = OracleODE(rx, kp)
        cd = {k: c0[s, a] for s, k in enumerate(t.species)}
        new, fl, cnt = ode.step(cd, 1.0, m2c[a])
        for s in range(t.n_dyn):
            ref = new[t.species[s]]
            assert abs(conc[s, a] - ref) <= 1e-6 * abs(ref) + 1e-12, (a, t.species[s])


def test_c_stencil_bitwise():
    z = np.load(os.path.join(GOLDEN, 'stencil.npz'))
    for shape in ('17x23', '64x64', '128x96'):
        for dt in (1.0, 5.0):
            f = np.ascontiguousarray(z['f0_' + shape].copy())
            cpu.diffuse(f, 5.0 * min(dt, 0.01), olat.n_substeps(dt))
            assert np.array_equal(f, z['f_%s_dt%g' % (shape, dt)])
