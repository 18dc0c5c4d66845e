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


@pytest.mark.parametrize('name', ['c2', 'c3kin', 'c5kin'])
def test_c_oracle_dp45_vs_odeint_trajectories(name):
    """The C oracle's DP45 (the GPU kernels' algorithm, rtol 1e-8) follows the
    committed odeint trajectories (tests/golden/make_odeint_traj.py) within the
    north-star 1e-6 relative + 1e-10 absolute, step after step; and the
    seeded colony generator still reproduces the fixture's inputs."""
    import sys
    sys.path.insert(0, GOLDEN)
    import make_odeint_traj as mk
    z = np.load(os.path.join(GOLDEN, '%s_odeint_traj.npz' % name))
    (_, n_agents, stride, _, steps, every) = mk.CASES[name]
    cfg, t, params, conc = mk._setup(name)
    sample = z['sample']
    assert np.array_equal(params[:, sample], z['params']) and np.array_equal(conc[:, sample], z['conc'])
    p = np.ascontiguousarray(z['params'])
    c = np.ascontiguousarray(z['conc'])
    m2c = np.full(c.shape[1], float(z['m2c']))
    h = np.zeros(c.shape[1])
    desc = cpu.Desc(t)
    k = 0
    for step in range(1, steps + 1):
        fl, _, st, _ = cpu.step_dopri5(desc, 1.0, p, c, m2c, h_state=h)
        assert not st.any()
        if step % every == 0:
            ref = z['y'][:, k]
            assert (np.abs(c[:t.n_dyn].T - ref) <= 1e-6 * np.abs(ref) + 1e-10).all(), step
            fr = z['flux'][:, k]
            assert (np.abs(fl.T - fr) <= 1e-6 * np.abs(fr) + 1e-10).all(), step
            k += 1
