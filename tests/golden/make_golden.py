"""Generate the committed golden fixtures (run once in the build container).

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Needs /root/reference (read-only, importable parts only) and scipy.  Writes:

* fluxes.json -- reference ``KineticFluxModel.get_fluxes`` outputs
  (vivarium/library/kinetic_rate_laws.py:240-297, imported from the reference
  tree) for: the reference's own toy network, get_glc_lct_config,
  get_glc_lct_transport, an enzyme-sharing aliasing case, a reversible
  reaction without kcat_r, zero-Km entries, and seeded random networks.
* convenience_kinetics_subset.csv -- rows of the reference fixture
  vivarium/reference_data/convenience_kinetics.csv (every 10th row + the
  first 5 + the last).
* stencil.npz -- scipy.ndimage.convolve(mode='reflect') diffusion
  (restating vivarium/processes/diffusion_field.py:385-394 around the real
  scipy convolve) on 17x23 / 64x64 / 128x96 fields for dt in {1, 5, 10}.

Nothing here is imported at test time; tests read only the written files.
"""

import csv
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(os.path.dirname(HERE))
sys.path.insert(0, REPO)
sys.path.insert(0, HERE)
sys.path.insert(0, '/root/reference')

from netcodec import encode_network, encode_conc  # noqa: E402

SEED = 20261015


def reference_fluxes(reactions, kinetics, concs):
    import copy
    from vivarium.library.kinetic_rate_laws import KineticFluxModel
    model = KineticFluxModel(copy.deepcopy(reactions), copy.deepcopy(kinetics))
    return [{k: float(v) for k, v in model.get_fluxes(c).items()} for c in concs]


def species_of(reactions, kinetics):
    keys = []
    for rid, spec in reactions.items():
        for m in spec['stoichiometry']:
            if m not in keys:
                keys.append(m)
        for e in spec['catalyzed by']:
            if e not in keys:
                keys.append(e)
    for rid, enz in kinetics.items():
        for e, params in enz.items():
            for p in params:
                if isinstance(p, tuple) and p not in keys:
                    keys.append(p)
    return keys


def random_concs(rng, keys, n):
    out = []
    for _ in range(n):
        c = {}
        for k in keys:
            c[k] = float(10 ** rng.uniform(-4, 1)) if rng.random() > 0.05 else 0.0
        out.append(c)
    return out


def random_network(rng, n_rx, n_mol, n_enz):
    ports = ['internal', 'external', 'periplasm']
    mols = [(ports[int(rng.integers(0, 3))], 'M%d' % i) for i in range(n_mol)]
    enzymes = [('internal', 'E%d' % i) for i in range(n_enz)]
    reactions = {}
    for r in range(n_rx):
        ns, npd = int(rng.integers(1, 4)), int(rng.integers(0, 3))
        pick = rng.choice(n_mol, ns + npd, replace=False)
        st = {mols[i]: -float(rng.integers(1, 3)) for i in pick[:ns]}
        st.update({mols[i]: float(rng.integers(1, 3)) for i in pick[ns:]})
        n_cat = min(int(rng.integers(1, 3)), n_enz)
        cat = [enzymes[i] for i in rng.choice(n_enz, n_cat, replace=False)]
        reactions['R%d' % r] = {'stoichiometry': st,
                                'is reversible': bool(rng.random() < 0.25),
                                'catalyzed by': cat}
    kinetics = {}
    for rid, spec in reactions.items():
        kinetics[rid] = {}
        for e in spec['catalyzed by']:
            if rng.random() < 0.1 and len(kinetics[rid]) == 0 and len(spec['catalyzed by']) > 1:
                continue  # enzyme without parameters: skipped by make_rate_laws
            # Km for every molecule of every reaction this enzyme catalyses
            mset = []
            for spec2 in reactions.values():
                if e in spec2['catalyzed by']:
                    for m in spec2['stoichiometry']:
                        if m not in mset:
                            mset.append(m)
            p = {}
            for m in mset:
                u = rng.random()
                p[m] = None if u < 0.15 else (0.0 if u < 0.2 else float(10 ** rng.uniform(-3, 1)))
            p['kcat_f'] = float(10 ** rng.uniform(-1, 3))
            kinetics[rid][e] = p
    return reactions, kinetics


def main():
    from lens_amd import configs
    from vivarium.library import kinetic_rate_laws as krl
    rng = np.random.default_rng(SEED)
    cases = []

    def add(name, reactions, kinetics, concs):
        fl = reference_fluxes(reactions, kinetics, concs)
        cases.append({'name': name, 'network': encode_network(reactions, kinetics),
                      'concs': [encode_conc(c) for c in concs], 'fluxes': fl})

    # the reference module's own toy data (kinetic_rate_laws.py:301-366)
    from vivarium.library.dict_utils import tuplify_port_dicts
    toy_conc = tuplify_port_dicts(krl.toy_initial_state)
    add('reference_toy', krl.toy_reactions, krl.toy_kinetics,
        [toy_conc] + random_concs(rng, list(toy_conc), 7))

    for name, cfg in (('glc_lct', configs.glc_lct_config()),
                      ('glc_lct_transport', configs.glc_lct_transport_config()),
                      ('toy', configs.toy_config()),
                      ('glc_ac', configs.glc_ac_config())):
        keys = species_of(cfg['reactions'], cfg['kinetic_parameters'])
        add(name, cfg['reactions'], cfg['kinetic_parameters'], random_concs(rng, keys, 16))

    # aliasing: enzyme E shared by R1, R2; R1 marks B non-limiting (None) which
    # strips B from the shared partition that R2's rate law also reads.
    ali_rx = {
        'R1': {'stoichiometry': {('internal', 'A'): -1, ('internal', 'B'): -1, ('internal', 'C'): 1},
               'is reversible': False, 'catalyzed by': [('internal', 'E')]},
        'R2': {'stoichiometry': {('internal', 'B'): -1, ('internal', 'D'): 1},
               'is reversible': False, 'catalyzed by': [('internal', 'E')]},
    }
    ali_kp = {
        'R1': {('internal', 'E'): {('internal', 'A'): 0.5, ('internal', 'B'): None, 'kcat_f': 10.0}},
        'R2': {('internal', 'E'): {('internal', 'A'): 0.5, ('internal', 'B'): 2.0, 'kcat_f': 3.0}},
    }
    add('aliasing', ali_rx, ali_kp, random_concs(rng, species_of(ali_rx, ali_kp), 16))

    # reversible without kcat_r: reverse set also uses kcat_f
    rev_rx = {'RV': {'stoichiometry': {('internal', 'A'): -1, ('external', 'B'): 1},
                     'is reversible': True, 'catalyzed by': [('internal', 'E')]}}
    rev_kp = {'RV': {('internal', 'E'): {('internal', 'A'): 0.3, ('external', 'B'): 0.7,
                                         'kcat_f': 4.0, 'kcat_r': 0}}}
    add('reversible', rev_rx, rev_kp, random_concs(rng, species_of(rev_rx, rev_kp), 16))

    # zero Km: cofactor_numerator -> 0, cofactor_denominator -> 1
    z_rx = {'RZ': {'stoichiometry': {('internal', 'A'): -1, ('internal', 'B'): -1, ('internal', 'C'): 1},
                   'is reversible': False, 'catalyzed by': [('internal', 'E')]},
            'RY': {'stoichiometry': {('internal', 'B'): -1, ('internal', 'D'): 1},
                   'is reversible': False, 'catalyzed by': [('internal', 'E')]}}
    z_kp = {'RZ': {('internal', 'E'): {('internal', 'A'): 0.0, ('internal', 'B'): 1.0, 'kcat_f': 2.0}},
            'RY': {('internal', 'E'): {('internal', 'A'): 1.5, ('internal', 'B'): 0, 'kcat_f': 5.0}}}
    add('zero_km', z_rx, z_kp, random_concs(rng, species_of(z_rx, z_kp), 16))

    for i in range(12):
        n_rx = int(rng.integers(2, 65))
        rx, kp = random_network(rng, n_rx, int(rng.integers(4, 40)), int(rng.integers(1, 12)))
        add('random_%02d' % i, rx, kp, random_concs(rng, species_of(rx, kp), 8))

    with open(os.path.join(HERE, 'fluxes.json'), 'w') as f:
        json.dump({'seed': SEED, 'source': 'vivarium.library.kinetic_rate_laws (reference)',
                   'cases': cases}, f, indent=None, separators=(',', ':'))

    # reference fixture subset
    src = '/root/reference/vivarium/reference_data/convenience_kinetics.csv'
    with open(src) as f:
        rows = list(csv.reader(f))
    header, body = rows[0], rows[1:]
    keep = sorted(set(list(range(5)) + list(range(0, len(body), 10)) + [len(body) - 1]))
    with open(os.path.join(HERE, 'convenience_kinetics_subset.csv'), 'w', newline='') as f:
        w = csv.writer(f)
        w.writerow(header)
        for i in keep:
            w.writerow(body[i])

    # stencil fixtures around the real scipy convolve
    from scipy.ndimage import convolve
    lap = np.array([[0.0, 1.0, 0.0], [1.0, -4.0, 1.0], [0.0, 1.0, 0.0]])
    out = {}
    for (nx, ny) in ((17, 23), (64, 64), (128, 96)):
        f0 = rng.random((nx, ny)) * 10 ** rng.uniform(-2, 2, (nx, ny))
        out['f0_%dx%d' % (nx, ny)] = f0
        coef = 5.0 / (1.0 * 1.0)   # diffusion / (dx*dy), bounds == n_bins
        for dt in (1.0, 5.0, 10.0):
            fn = f0.copy()
            t = 0.0
            sub = min(dt, 0.01)
            n = 0
            while t < dt:
                fn += coef * sub * convolve(fn, lap, mode='reflect')
                t += sub
                n += 1
            out['f_%dx%d_dt%g' % (nx, ny, dt)] = f0 + (fn - f0)
            out['n_%dx%d_dt%g' % (nx, ny, dt)] = np.array(n)
    np.savez_compressed(os.path.join(HERE, 'stencil.npz'), **out)
    print('wrote', len(cases), 'flux cases')


def colony_metrics_fixture():
    """colony_metrics_subset.npz from vivarium/reference_data/colony_metrics.csv
    (the reference's division / phylogeny golden): for each of the 30 agent ids
    its number of emitted rows (lifetime; later-born agents' columns are padded
    from row 0, vivarium/library/timeseries.py:53-69) and the mass, volume,
    width, length, surface_area, protein values at every 10th row plus the
    first and last three rows of its life."""
    src = '/root/reference/vivarium/reference_data/colony_metrics.csv'
    with open(src) as f:
        rows = list(csv.reader(f))
    header, body = rows[0], rows[1:]
    cols = {tuple(h.split(',')[1:]): i for i, h in enumerate(header)}
    ids = []
    for h in header:
        parts = h.split(',')
        if parts[0] == 'agents' and parts[1] not in ids:
            ids.append(parts[1])
    variables = ('mass', 'volume', 'width', 'length', 'surface_area', 'protein')
    out = {'ids': np.array(ids), 'variables': np.array(variables)}
    for aid in ids:
        series = []
        for v in variables:
            i = cols[(aid, 'internal' if v == 'protein' else 'boundary', v)]
            series.append([float(r[i]) for r in body if r[i] != ''])
        n = len(series[0])
        keep = sorted(set(list(range(0, n, 10)) + [0, 1, 2, n - 3, n - 2, n - 1]))
        out['n_' + aid] = np.array(n)
        out['k_' + aid] = np.array(keep)
        out['v_' + aid] = np.array([[series[j][k] for j in range(len(variables))] for k in keep])
    np.savez_compressed(os.path.join(HERE, 'colony_metrics_subset.npz'), **out)
    # and the file itself (data: the emitter test rebuilds it byte for byte)
    import gzip
    with open(src, 'rb') as f, gzip.open(os.path.join(HERE, 'colony_metrics.csv.gz'), 'wb', 9) as g:
        g.write(f.read())
    print('wrote colony_metrics_subset.npz + colony_metrics.csv.gz:', len(ids), 'agents')


if __name__ == '__main__':
    if '--colony-metrics' in sys.argv:
        colony_metrics_fixture()
    else:
        main()
        colony_metrics_fixture()
