"""Network configurations and synthetic colony generators.

The dictionaries are in the reference's ConvenienceKinetics configuration
schema (``reactions`` / ``kinetic_parameters`` / ``initial_state`` /
``ports``), so any reference config drops straight in.

* :func:`glc_lct_config` -- get_glc_lct_config (vivarium/processes/convenience_kinetics.py:448-524),
  the network the reference fixture convenience_kinetics.csv is produced with.
* :func:`glc_lct_transport_config` -- get_glc_lct_transport (:357-445).
* :func:`toy_config` -- get_toy_config (:527-571).
* :func:`glc_ac_config` -- glucose uptake + a synthetic acetate secretion
  (BASELINE configs 3-4; SURVEY.md §8d C3: no acetate reaction exists in
  the reference, so this one is ours, written in the reference schema).
* :func:`heterogeneous_colony` -- SURVEY.md §8d C2 distributions.
* :func:`synthetic_network` -- SURVEY.md §8d C5-style random network.
"""

from __future__ import annotations

import copy
import math

import numpy as np

SEED = 20261015


def glc_lct_config():
    reactions = {
        'EX_glc__D_e': {
            'stoichiometry': {
                ('internal', 'g6p_c'): 1.0,
                ('external', 'glc__D_e'): -1.0,
                ('internal', 'pep_c'): -1.0,
                ('internal', 'pyr_c'): 1.0,
            },
            'is reversible': False,
            'catalyzed by': [('internal', 'EIIglc')],
        },
        'EX_lcts_e': {
            'stoichiometry': {
                ('external', 'lcts_e'): -1.0,
                ('internal', 'lcts_p'): 1.0,
            },
            'is reversible': False,
            'catalyzed by': [('internal', 'LacY')],
        },
    }
    kinetics = {
        'EX_glc__D_e': {
            ('internal', 'EIIglc'): {
                ('external', 'glc__D_e'): 1e0,
                ('internal', 'pep_c'): None,
                'kcat_f': 6e1,
            }
        },
        'EX_lcts_e': {
            ('internal', 'LacY'): {
                ('external', 'lcts_e'): 1e0,
                'kcat_f': 6e1,
            }
        },
    }
    initial_state = {
        'internal': {
            'EIIglc': 1.8e-3, 'g6p_c': 0.0, 'pep_c': 1.8e-1,
            'pyr_c': 0.0, 'LacY': 0, 'lcts_p': 0.0,
        },
        'external': {'glc__D_e': 10.0, 'lcts_e': 10.0},
    }
    ports = {
        'internal': ['g6p_c', 'pep_c', 'pyr_c', 'EIIglc', 'LacY', 'lcts_p'],
        'external': ['glc__D_e', 'lcts_e'],
    }
    return {'reactions': reactions, 'kinetic_parameters': kinetics,
            'initial_state': initial_state, 'ports': ports}


def glc_lct_transport_config():
    reactions = {
        'LCTSt3ipp': {
            'stoichiometry': {
                ('internal', 'h_c'): 1.0, ('external', 'h_p'): -1.0,
                ('internal', 'lcts_c'): 1.0, ('external', 'lcts_p'): -1.0},
            'is reversible': False,
            'catalyzed by': [('internal', 'LacY')]},
        'GLCptspp': {
            'stoichiometry': {
                ('internal', 'g6p_c'): 1.0, ('external', 'glc__D_e'): -1.0,
                ('internal', 'pep_c'): -1.0, ('internal', 'pyr_c'): 1.0},
            'is reversible': False,
            'catalyzed by': [('internal', 'EIIglc')]},
        'GLCt2pp': {
            'stoichiometry': {
                ('internal', 'glc__D_c'): 1.0, ('external', 'glc__D_p'): -1.0,
                ('internal', 'h_c'): 1.0, ('external', 'h_p'): -1.0},
            'is reversible': False,
            'catalyzed by': [('internal', 'GalP')]},
    }
    kinetics = {
        'LCTSt3ipp': {('internal', 'LacY'): {
            ('external', 'h_p'): None, ('external', 'lcts_p'): 1e0, 'kcat_f': 7.8e2}},
        'GLCptspp': {('internal', 'EIIglc'): {
            ('external', 'glc__D_e'): 1e0, ('internal', 'pep_c'): 1e0, 'kcat_f': 7.5e4}},
        'GLCt2pp': {('internal', 'GalP'): {
            ('external', 'glc__D_p'): 1e0, ('external', 'h_p'): None, 'kcat_f': 1.5e2}},
    }
    initial_state = {
        'internal': {'EIIglc': 1.8e-3, 'g6p_c': 0.0, 'pep_c': 1.8e-1,
                     'pyr_c': 0.0, 'LacY': 0, 'lcts_p': 0.0},
        'external': {'glc__D_e': 10.0, 'lcts_e': 10.0},
    }
    return {'reactions': reactions, 'kinetic_parameters': kinetics,
            'initial_state': initial_state}


def toy_config():
    return {
        'reactions': {'reaction1': {
            'stoichiometry': {('internal', 'A'): 1, ('external', 'B'): -1},
            'is reversible': False,
            'catalyzed by': [('internal', 'enzyme1')]}},
        'kinetic_parameters': {'reaction1': {('internal', 'enzyme1'): {
            ('external', 'B'): 0.2, 'kcat_f': 5e1}}},
        'initial_state': {'internal': {'A': 1.0, 'enzyme1': 1e-1},
                          'external': {'B': 10.0}},
        'ports': {'internal': ['A', 'enzyme1'], 'external': ['B']},
    }


def glc_ac_config():
    """Glucose PTS uptake (glc_lct's EX_glc__D_e) + acetate overflow secretion."""
    cfg = glc_lct_config()
    reactions = {'EX_glc__D_e': cfg['reactions']['EX_glc__D_e']}
    kinetics = {'EX_glc__D_e': cfg['kinetic_parameters']['EX_glc__D_e']}
    reactions['EX_ac_e'] = {
        'stoichiometry': {('internal', 'g6p_c'): -1.0, ('external', 'ac_e'): 2.0},
        'is reversible': False,
        'catalyzed by': [('internal', 'AckA')],
    }
    kinetics['EX_ac_e'] = {('internal', 'AckA'): {('internal', 'g6p_c'): 5e-1, 'kcat_f': 2e1}}
    initial_state = {
        'internal': {'EIIglc': 1.8e-3, 'g6p_c': 0.0, 'pep_c': 1.8e-1, 'pyr_c': 0.0,
                     'AckA': 1.0e-3},
        'external': {'glc__D_e': 10.0, 'ac_e': 0.0},
    }
    return {'reactions': reactions, 'kinetic_parameters': kinetics,
            'initial_state': initial_state}


# ---------------------------------------------------------------------------
# colony generators (SoA numpy; the engine uploads them)
# ---------------------------------------------------------------------------

def initial_conc(table, initial_state, n_agents):
    """[n_species, n] float64 from a reference initial_state dict (missing -> 0)."""
    conc = np.zeros((table.n_species, n_agents), dtype=np.float64)
    for s, (port, name) in enumerate(table.species):
        conc[s, :] = float(initial_state.get(port, {}).get(name, 0.0))
    return conc


def heterogeneous_colony(table, config, n_agents, seed=SEED, sigma=0.25):
    """per-agent kcat/Km x lognormal(0, sigma); EIIglc ~ U(0.9,2.7)e-3,
    LacY ~ U(0, 2e-3); internal x U(0.5,1.5); glc__D_e ~ U(0.1,10), lcts_e ~ U(0,10)."""
    rng = np.random.default_rng(seed)
    params = np.repeat(table.param_defaults[:, None], n_agents, axis=1)
    params = params * rng.lognormal(0.0, sigma, size=params.shape)
    conc = initial_conc(table, config['initial_state'], n_agents)
    for s, (port, name) in enumerate(table.species):
        if port == 'external':
            continue
        conc[s] *= rng.uniform(0.5, 1.5, n_agents)
    draws = {
        ('internal', 'EIIglc'): lambda: rng.uniform(0.9e-3, 2.7e-3, n_agents),
        ('internal', 'LacY'): lambda: rng.uniform(0.0, 2e-3, n_agents),
        ('external', 'glc__D_e'): lambda: rng.uniform(0.1, 10.0, n_agents),
        ('external', 'lcts_e'): lambda: rng.uniform(0.0, 10.0, n_agents),
    }
    for key, draw in draws.items():
        if key in table.species:
            conc[table.species.index(key)] = draw()
    return np.ascontiguousarray(params), np.ascontiguousarray(conc)


def gaussian_bump_field(n_bins, base=10.0, amp=5.0, sigma_frac=0.125):
    nx, ny = n_bins
    x = (np.arange(nx) + 0.5)[:, None] - nx / 2
    y = (np.arange(ny) + 0.5)[None, :] - ny / 2
    sig = sigma_frac * min(nx, ny)
    return base + amp * np.exp(-(x * x + y * y) / (2 * sig * sig))


def synthetic_network(n_species=50, n_reactions=40, n_enzymes=10, seed=SEED,
                      n_external=4):
    """C5-style random network in the reference schema: irreversible reactions
    with 1-3 substrates and 1-2 products, Km log-U[1e-3, 1e1], kcat log-U[1e-1, 1e4]."""
    rng = np.random.default_rng(seed)
    internal = [('internal', 'm%02d' % i) for i in range(n_species - n_external)]
    external = [('external', 'x%02d' % i) for i in range(n_external)]
    mols = internal + external
    enzymes = [('internal', 'E%02d' % i) for i in range(n_enzymes)]
    reactions, kinetics = {}, {}
    for r in range(n_reactions):
        rid = 'R%03d' % r
        ns = int(rng.integers(1, 4))
        npd = int(rng.integers(1, 3))
        pick = rng.choice(len(mols), ns + npd, replace=False)
        subs = [mols[i] for i in pick[:ns]]
        prods = [mols[i] for i in pick[ns:]]
        st = {m: -float(rng.integers(1, 3)) for m in subs}
        st.update({m: float(rng.integers(1, 3)) for m in prods})
        enz = enzymes[int(rng.integers(0, n_enzymes))]
        reactions[rid] = {'stoichiometry': st, 'is reversible': False, 'catalyzed by': [enz]}
        p = {m: float(10 ** rng.uniform(-3, 1)) for m in subs}
        p['kcat_f'] = float(10 ** rng.uniform(-1, 4))
        kinetics[rid] = {enz: p}
    # an enzyme's partition holds the substrates of every reaction it catalyses
    # (kinetic_rate_laws.py:84-95), so each of its rate laws needs their Kms
    for rid, spec in reactions.items():
        enz = spec['catalyzed by'][0]
        p = kinetics[rid][enz]
        for other in reactions.values():
            if enz in other['catalyzed by']:
                for m, c in other['stoichiometry'].items():
                    if c < 0 and m not in p:
                        p[m] = float(10 ** rng.uniform(-3, 1))
    initial = {'internal': {k[1]: float(rng.uniform(0.1, 2.0)) for k in internal},
               'external': {k[1]: float(rng.uniform(1.0, 10.0)) for k in external}}
    for e in enzymes:
        initial['internal'][e[1]] = float(10 ** rng.uniform(-4, -2))
    return {'reactions': reactions, 'kinetic_parameters': kinetics, 'initial_state': initial}


def deepcopy_config(cfg):
    return copy.deepcopy(cfg)
