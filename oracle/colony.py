"""Oracle for growth, derivers and division -- TEST INFRASTRUCTURE ONLY.

Restates, per agent and per timestep, what the reference does around the
kinetics when cells grow and divide:

* ``GrowthProtein.next_update`` (vivarium/processes/growth_protein.py:88-107):
  ``total = p*exp(r*dt)``, ``new = int(total - p)``, ``+1`` if ``u < total -
  int(total)`` with ``u = np.random.random()``; ``divide = p >= 2*p0`` on the
  step-start protein.
* ``Growth.next_update`` (vivarium/processes/growth.py:101-107): ``mass*exp(r*dt)``.
* ``DivisionVolume.next_update`` (vivarium/processes/division_volume.py:39-45):
  ``divide = volume >= 2.4 fL`` on the step-start volume.
* ``TreeMass`` (vivarium/processes/tree_mass.py:10-18, 55-64):
  ``mass = 0 fg + mw*(count/N_A)``, the g -> fg conversion done by pint as
  ``x * (1/1e-15)``.
* ``DeriveGlobals.next_update`` (vivarium/processes/derive_globals.py:131-152):
  ``volume = mass/density`` (pint's fg*L/g -> fL factor evaluates to
  1.0000000000000002), ``mmol_to_counts = N_A*volume`` in L/mmol, capsule
  ``length`` and ``surface_area`` (:20-50) from the *unconverted* magnitude.
* ``MetaDivision`` (vivarium/processes/meta_division.py:60-88) +
  ``Store.apply_update`` ``_divide`` (vivarium/core/experiment.py:664-697):
  daughters ``id+'0'``, ``id+'1'`` appended after the other agents in mother
  order, mother deleted; dividers (vivarium/core/registry.py:197-280): floats
  ``split`` (halved), nodes without a divider copied, ``divide`` flag reset.

Order inside one step (Experiment.update, experiment.py:1365-1446): every
process computes from the step-start state, updates are applied, then the
derivers run in store order -- mass_deriver, globals_deriver, division -- so a
mother is split with its post-growth, re-derived values and the daughters'
derivers first run on the next step.

``replay_colony_metrics`` reproduces vivarium/reference_data/colony_metrics.csv
(growth_division_minimal agents, growth_rate 0.001, np.random.seed(1)); the
uniform draws are numpy's MT19937 stream in the reference's consumption order
(two draws taken during setup, then one per agent per step in agent order).
"""

from __future__ import annotations

import math
from typing import Dict, List

import numpy as np

N_A = 6.022140857e23          # scipy<1.4 constant the fixtures were made with
PI = math.pi
FG_PER_G = 1 / 1e-15          # pint's g -> fg factor, as evaluated (999999999999999.9)
VOLUME_TO_FL = 1e-18 / 1e-3 * 1e18 * 1e-3   # pint's fg*L/g -> fL factor (1.0000000000000002)
DENSITY = 1100.0              # g/L
PROTEIN_MW = 2.09e4           # g/mol
INITIAL_MASS_FG = 1339.0


def initial_protein(initial_mass_fg=INITIAL_MASS_FG, mw=PROTEIN_MW, avogadro=N_A):
    """growth_protein.py:46-47: initial_mass.to('g') / mw * N_A."""
    return initial_mass_fg * 1e-15 / mw * avogadro


def tree_mass(protein, mw=PROTEIN_MW, avogadro=N_A):
    return 0.0 + (mw * (protein / avogadro)) * FG_PER_G


def length_from_volume(volume, width):
    radius = width / 2
    cylinder_length = (volume - (4 / 3) * PI * radius ** 3) / (PI * radius ** 2)
    return cylinder_length + 2 * radius


def surface_area_from_length(length, width):
    radius = width / 2
    cylinder_length = length - width
    return 3 * PI * radius ** 2 + 2 * PI * radius * cylinder_length


def derive_globals(mass, width=1.0, density=DENSITY, avogadro=N_A):
    """Returns (volume fL, mmol_to_counts L/mmol, length um, surface_area um^2)."""
    vol = mass / density
    length = length_from_volume(vol, width)
    return vol * VOLUME_TO_FL, avogadro * (vol * 1e-15) * 1e-3, length, surface_area_from_length(length, width)


def growth_protein_step(protein, factor, u, divide_protein):
    total = protein * factor
    new = int(total - protein)
    extra = total - int(total)
    if u < extra:
        new += 1
    return protein + new, protein >= divide_protein


VARS = ('mass', 'volume', 'width', 'length', 'surface_area', 'protein')


def replay_colony_metrics(n_steps=2400, growth_rate=0.001, seed=1, setup_draws=2,
                          roots=('0', '1')) -> Dict[str, Dict[str, List[float]]]:
    """Dict-per-agent replay (the reference's structure) of colony_metrics.csv:
    returns {agent_id: {var: [value per emitted step of that agent]}}."""
    rs = np.random.RandomState(seed)
    rs.random_sample(setup_draws)
    p0 = initial_protein()
    factor = np.exp(growth_rate * 1.0)
    agents = []
    for rid in roots:
        mass = tree_mass(p0)
        vol, m2c, length, sa = derive_globals(mass)
        agents.append({'id': rid, 'protein': p0, 'mass': mass, 'volume': vol, 'width': 1.0,
                       'length': length, 'surface_area': sa, 'divide': False})
    hist: Dict[str, Dict[str, List[float]]] = {}

    def emit():
        for a in agents:
            h = hist.setdefault(a['id'], {v: [] for v in VARS})
            for v in VARS:
                h[v].append(a[v])

    emit()
    for _ in range(n_steps):
        # processes: GrowthProtein from the step-start state, one draw per agent
        for a in agents:
            a['protein'], a['divide'] = growth_protein_step(a['protein'], factor, rs.random_sample(),
                                                            2 * p0)
        # derivers in store order: mass, globals, division
        survivors, daughters = [], []
        for a in agents:
            a['mass'] = tree_mass(a['protein'])
            raw = a['mass'] / DENSITY
            a['volume'] = raw * VOLUME_TO_FL
            a['length'] = length_from_volume(raw, a['width'])
            a['surface_area'] = surface_area_from_length(a['length'], a['width'])
            if a['divide']:
                for k in '01':
                    d = dict(a)
                    d['id'] = a['id'] + k
                    for v in ('protein', 'mass', 'volume', 'length', 'surface_area'):
                        d[v] = a[v] / 2
                    d['divide'] = False
                    daughters.append(d)
            else:
                survivors.append(a)
        agents = survivors + daughters
        emit()
    return hist


# ---------------------------------------------------------------------------
# SoA restatement (the device pipeline's layout), for random colonies
# ---------------------------------------------------------------------------

def soa_step(cell, ids, model, dt, u=None, rate=0.001, division_volume=2.4, divide_protein=None,
             width=1.0):
    """One step on SoA numpy arrays.

    cell: dict of float64 arrays (mass, volume, length, surface_area, protein,
    m2c, angle, x, y) -- each [n]; ids: list of str.  model: 'growth_protein'
    or 'growth' (+ DivisionVolume).  Returns (cell', ids', order) where order[j]
    is the source agent of new agent j (mothers appear twice)."""
    n = len(ids)
    factor = np.exp(rate * dt)
    if model == 'growth_protein':
        p = cell['protein'].copy()
        div = np.zeros(n, dtype=bool)
        for a in range(n):
            p[a], div[a] = growth_protein_step(cell['protein'][a], factor, u[a], divide_protein)
        cell = dict(cell, protein=p)
        mass = np.array([tree_mass(x) for x in p])
    else:
        div = cell['volume'] >= division_volume
        mass = cell['mass'] * factor
    raw = mass / DENSITY
    length = np.array([length_from_volume(v, width) for v in raw])
    cell = dict(cell, mass=mass, volume=raw * VOLUME_TO_FL, m2c=N_A * (raw * 1e-15) * 1e-3, length=length,
                surface_area=np.array([surface_area_from_length(x, width) for x in length]))
    keep = np.flatnonzero(~div)
    moth = np.flatnonzero(div)
    order = np.concatenate([keep, np.repeat(moth, 2)]).astype(np.int64)
    out = {k: v[order].copy() for k, v in cell.items()}
    nk = len(keep)
    for v in ('mass', 'volume', 'length', 'surface_area', 'protein'):
        if v in out:
            out[v][nk:] = out[v][nk:] / 2
    if 'x' in out:
        for j in range(len(moth)):
            for k, ratio in enumerate((-0.25, 0.25)):
                a = nk + 2 * j + k
                out['x'][a] = out['x'][a] + out['length'][a] * 2 * ratio * math.cos(out['angle'][a])
                out['y'][a] = out['y'][a] + out['length'][a] * 2 * ratio * math.sin(out['angle'][a])
    new_ids = [ids[a] for a in keep] + [ids[a] + k for a in moth for k in '01']
    return out, new_ids, order


def philox_uniform(seed, step, root, depth, path):
    """Philox4x32-10 uniform with the device's counter / key layout
    (lens_amd/csrc/vk_cells.hip: philox_uniform)."""
    m32 = 0xFFFFFFFF
    path &= 0xFFFFFFFFFFFFFFFF
    c = [step & m32, root & m32, path & m32, (path >> 32) & m32]
    k = [(seed + depth) & m32, (seed >> 32) & m32]
    for r in range(10):
        if r:
            k = [(k[0] + 0x9E3779B9) & m32, (k[1] + 0xBB67AE85) & m32]
        p0 = 0xD2511F53 * c[0]
        p1 = 0xCD9E8D57 * c[2]
        c = [((p1 >> 32) ^ c[1] ^ k[0]) & m32, p1 & m32, ((p0 >> 32) ^ c[3] ^ k[1]) & m32, p0 & m32]
    return ((c[0] >> 5) * 67108864.0 + (c[1] >> 6)) / 9007199254740992.0
