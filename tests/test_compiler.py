"""Host logic: the rate-law compiler reproduces the reference's rate laws."""

import numpy as np
import pytest

from netcodec import decode_network, decode_conc
from table_eval import table_fluxes, table_euler
from lens_amd.rate_law_compiler import compile_rate_laws
from lens_amd.configs import glc_lct_config
from oracle.kinetics import OracleAgent, mmol_to_counts


def _conc_vec(t, conc):
    return np.array([float(conc.get(k, 0.0)) for k in t.species])


def test_compiled_table_reproduces_reference_fluxes_bitwise(golden_fluxes):
    for case in golden_fluxes['cases']:
        rx, kp = decode_network(case['network'])
        t = compile_rate_laws(rx, kp)
        assert t.reaction_ids == list(case['fluxes'][0].keys())
        for conc_items, expect in zip(case['concs'], case['fluxes']):
            got = table_fluxes(t, _conc_vec(t, decode_conc(conc_items)), t.param_defaults)
            assert got.tolist() == [expect[r] for r in t.reaction_ids], case['name']


def test_glc_lct_layout():
    cfg = glc_lct_config()
    t = compile_rate_laws(cfg['reactions'], cfg['kinetic_parameters'])
    assert t.species[:t.n_dyn] == [('internal', 'g6p_c'), ('internal', 'pep_c'),
                                   ('internal', 'pyr_c'), ('internal', 'lcts_p')]
    assert t.external_ids == ['glc__D_e', 'lcts_e']
    assert t.reaction_ids == ['EX_glc__D_e', 'EX_lcts_e']
    # pep_c's Km is None -> removed from both numerator and partition
    assert ('internal', 'pep_c') not in [t.species[s] for s in t.mem_species]
    assert t.n_params == 4
    assert t.flops_rhs() > 0


def test_aliasing_is_replayed():
    rx = {
        'R1': {'stoichiometry': {('internal', 'A'): -1, ('internal', 'B'): -1, ('internal', 'C'): 1},
               'is reversible': False, 'catalyzed by': [('internal', 'E')]},
        'R2': {'stoichiometry': {('internal', 'B'): -1, ('internal', 'D'): 1},
               'is reversible': False, 'catalyzed by': [('internal', 'E')]},
    }
    kp = {'R1': {('internal', 'E'): {('internal', 'A'): 0.5, ('internal', 'B'): None, 'kcat_f': 10.0}},
          'R2': {('internal', 'E'): {('internal', 'A'): 0.5, ('internal', 'B'): 2.0, 'kcat_f': 3.0}}}
    t = compile_rate_laws(rx, kp)
    # R2's own cofactor set [B] keeps B; the shared partition lost B: [[A], [B]] -> [[A], []]
    l2 = 1
    den_sets = [[t.species[t.mem_species[m]] for m in range(t.set_ptr[s], t.set_ptr[s + 1])]
                for s in range(t.rl_den_ptr[l2], t.rl_den_ptr[l2 + 1])]
    assert den_sets == [[('internal', 'A')], [('internal', 'B')]] or \
        den_sets == [[('internal', 'A')], []]


def test_errors_mirror_reference():
    rx = {'R': {'stoichiometry': {('internal', 'A'): -1}, 'is reversible': False,
                'catalyzed by': [('internal', 'E')]}}
    with pytest.raises(NameError):
        compile_rate_laws(rx, {'R': {('internal', 'E'): {('internal', 'A'): 1.0,
                                                         'kcat_f': 1.0, 'kcat_r': 1.0}}})
    with pytest.raises(KeyError):
        compile_rate_laws(rx, {'Q': {}})
    with pytest.raises(KeyError):   # missing Km for a partition member
        compile_rate_laws(rx, {'R': {('internal', 'E'): {'kcat_f': 1.0}}})


def test_euler_table_matches_oracle_agent(golden_fluxes):
    rng = np.random.default_rng(3)
    for case in golden_fluxes['cases']:
        rx, kp = decode_network(case['network'])
        t = compile_rate_laws(rx, kp)
        agent = OracleAgent(rx, kp)
        m2c = mmol_to_counts()
        for conc_items in case['concs'][:4]:
            conc = decode_conc(conc_items)
            states = {}
            for (port, name), v in conc.items():
                states.setdefault(port, {})[name] = v
            dt = float(rng.choice([0.5, 1.0, 2.0]))
            fl, deltas, counts = agent.next_update(dt, states, m2c)
            cv = _conc_vec(t, conc)
            new, flux, cnt = table_euler(t, cv, t.param_defaults, dt, m2c)
            for s in range(t.n_dyn):
                port, name = t.species[s]
                assert new[s] == cv[s] + deltas[port][name]
            assert cnt.tolist() == [counts[e] for e in t.external_ids]
