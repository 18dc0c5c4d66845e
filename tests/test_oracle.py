"""The oracle, pinned against the reference's own fixtures and golden vectors."""

import csv
import os

import numpy as np
import pytest

from netcodec import decode_network, decode_conc
from oracle.rate_laws import OracleFluxModel
from oracle.kinetics import replay_single_agent, N_A_LEGACY, N_A_CODATA2018
from oracle import lattice as olat
from lens_amd.configs import glc_lct_config

GOLDEN = os.path.join(os.path.dirname(__file__), 'golden')


def test_oracle_matches_reference_fluxes_bitwise(golden_fluxes):
    n = 0
    for case in golden_fluxes['cases']:
        rx, kp = decode_network(case['network'])
        model = OracleFluxModel(rx, kp)
        for conc_items, expect in zip(case['concs'], case['fluxes']):
            got = model.get_fluxes(decode_conc(conc_items))
            assert list(got) == list(expect), case['name']
            for rid in expect:
                assert float(got[rid]) == expect[rid], (case['name'], rid)
                n += 1
    assert n > 500


def test_reference_toy_known_answer(golden_fluxes):
    # kinetic_rate_laws.test_kinetics (kinetic_rate_laws.py:369-374) on toy data
    case = [c for c in golden_fluxes['cases'] if c['name'] == 'reference_toy'][0]
    assert case['fluxes'][0] == {'ABC-13-RXN': 0.999000999000999,
                                 'TRANS-RXN-122': 1.9979820181818162}


def test_kcat_r_raises_like_reference():
    rx = {'R': {'stoichiometry': {('internal', 'A'): -1}, 'is reversible': True,
                'catalyzed by': [('internal', 'E')]}}
    kp = {'R': {('internal', 'E'): {('internal', 'A'): 1.0, 'kcat_f': 1.0, 'kcat_r': 2.0}}}
    with pytest.raises(NameError):
        OracleFluxModel(rx, kp)


def _fixture_rows():
    with open(os.path.join(GOLDEN, 'convenience_kinetics_subset.csv')) as f:
        return list(csv.DictReader(f))


def test_c1_replay_matches_reference_csv():
    """convenience_kinetics.csv (2521 rows) reproduced with N_A = 6.022140857e23.

    Internal species: <= 1e-14 relative.  External: <= 1e-15 mM absolute (the
    reference's pint unit conversion orders the count->mM arithmetic
    differently in the last bit; the per-step deltas are ~1e-2 mM)."""
    cfg = glc_lct_config()
    out = replay_single_agent(cfg['reactions'], cfg['kinetic_parameters'],
                              cfg['initial_state'], 2520)
    rows = _fixture_rows()
    for row in rows:
        t = int(float(row['time']))
        for k, v in out[t]['internal'].items():
            ref = float(row['internal_' + k])
            assert abs(v - ref) <= 1e-14 * abs(ref), (t, k, v, ref)
        for k, v in out[t]['external'].items():
            ref = float(row['external_' + k])
            assert abs(v - ref) <= 1e-15, (t, k, v, ref)


def test_c1_sensitivity_to_avogadro():
    # SURVEY.md §0 finding 2: today's N_A visibly breaks the fixture
    cfg = glc_lct_config()
    out = replay_single_agent(cfg['reactions'], cfg['kinetic_parameters'],
                              cfg['initial_state'], 600, avogadro=N_A_CODATA2018)
    rows = [r for r in _fixture_rows() if float(r['time']) == 600.0]
    ref = float(rows[0]['internal_g6p_c'])
    assert abs(out[600]['internal']['g6p_c'] - ref) > 1e-9 * abs(ref)


def test_stencil_oracle_matches_scipy_convolve_bitwise():
    z = np.load(os.path.join(GOLDEN, 'stencil.npz'))
    for shape in ('17x23', '64x64', '128x96'):
        f0 = z['f0_' + shape]
        nx, ny = f0.shape
        for dt in (1.0, 5.0, 10.0):
            key = '%s_dt%g' % (shape, dt)
            assert olat.n_substeps(dt) == int(z['n_' + key])
            got = olat.diffuse(f0, dt, 5.0, (nx, ny), (float(nx), float(ny)))
            assert np.array_equal(got, z['f_' + key]), key


def test_substep_counts_quirk():
    assert [olat.n_substeps(dt) for dt in (1.0, 5.0, 10.0)] == [100, 501, 1001]


def test_uniform_field_skip():
    f = np.full((8, 9), 3.25)
    assert np.array_equal(olat.diffuse(f, 1.0, 5.0, (8, 9), (8.0, 9.0)), f)
